// Host ingest check (include/nlp/ingest.hxx): the experiment's input
// preparation, written in oracle/ref_driver's `ingest` output format so the
// tests can compare it with the reference's own ingest byte for byte.
//   ingest_main <mtx> <seed> <d> <out_prefix> [symmetric_input]
//     -> <out_prefix>.csr  (u64 span, u64 M, u64 off[span+1], u32 keys[M])
//        <out_prefix>.del  (u64 n, u32 pairs[2n])
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include "nlp/ingest.hxx"

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: ingest_main <mtx> <seed> <d> <out_prefix> [symmetric_input]\n");
    return 2;
  }
  std::default_random_engine rnd((unsigned)strtoul(argv[2], nullptr, 10));
  const double d = atof(argv[3]);
  const bool sym = argc > 5 && atoi(argv[5]) != 0;
  nlp::Experiment ex = nlp::ingestExperiment(argv[1], sym, d, rnd);
  const std::string out = argv[4];
  FILE* f = fopen((out + ".csr").c_str(), "wb");
  if (!f) return 1;
  uint64_t S = ex.y.span(), M = ex.y.size();
  fwrite(&S, 8, 1, f);
  fwrite(&M, 8, 1, f);
  fwrite(ex.y.off.data(), 8, ex.y.off.size(), f);
  if (M) fwrite(ex.y.keys.data(), 4, M, f);
  fclose(f);
  f = fopen((out + ".del").c_str(), "wb");
  if (!f) return 1;
  uint64_t n = ex.deletions.size();
  fwrite(&n, 8, 1, f);
  for (auto& e : ex.deletions) {
    fwrite(&e.first, 4, 1, f);
    fwrite(&e.second, 4, 1, f);
  }
  fclose(f);
  printf("order %zu size %zu span %zu deletions %zu (x: size %zu)\n", ex.y.span() - 1, ex.y.size(), ex.y.span(),
         ex.deletions.size(), ex.x.size());
  return 0;
}
