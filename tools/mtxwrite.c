/* mtxwrite.c -- binary (u32 src, u32 dst) pairs -> MatrixMarket coordinate
 * pattern general text, for the batch timing tool (tools/batch_all.py): the
 * reference's main.cxx and nlp_main read the graph as an .mtx file
 * (main.cxx:190-200).  Usage: mtxwrite <pairs.bin> <n> <out.mtx>
 * pairs.bin = u32 src[m] then u32 dst[m] (m from the file size). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int main(int argc, char** argv) {
  if (argc != 4) { fprintf(stderr, "usage: mtxwrite <pairs.bin> <n> <out.mtx>\n"); return 2; }
  FILE* f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 1; }
  fseek(f, 0, SEEK_END);
  const long bytes = ftell(f);
  fseek(f, 0, SEEK_SET);
  const size_t m = (size_t)bytes / 8;
  uint32_t* p = (uint32_t*)malloc((size_t)bytes);
  if (!p || fread(p, 1, (size_t)bytes, f) != (size_t)bytes) { fprintf(stderr, "read failed\n"); return 1; }
  fclose(f);
  const unsigned long long n = strtoull(argv[2], NULL, 10);
  FILE* o = fopen(argv[3], "w");
  if (!o) { perror(argv[3]); return 1; }
  static char buf[1 << 22];
  setvbuf(o, buf, _IOFBF, sizeof buf);
  fprintf(o, "%%%%MatrixMarket matrix coordinate pattern general\n%llu %llu %zu\n", n, n, m);
  char line[32];
  for (size_t i = 0; i < m; ++i) {
    /* two decimal ids per line, written without printf */
    char* q = line + sizeof line;
    *--q = '\n';
    uint32_t x = p[m + i];
    do { *--q = (char)('0' + x % 10); x /= 10; } while (x);
    *--q = ' ';
    x = p[i];
    do { *--q = (char)('0' + x % 10); x /= 10; } while (x);
    fwrite(q, 1, (size_t)(line + sizeof line - q), o);
  }
  fclose(o);
  free(p);
  return 0;
}
