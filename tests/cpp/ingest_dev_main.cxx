// Device ingest check (nlp_main's route, SURVEY §8(f) N1 + N2): the file's pairs
// parsed on all threads (nlp::readMtxPairs), then nlp_dcsr_ingest and one
// nlp_dcsr_delete_batch of size_t(d * |E| / 2) with default_random_engine(seed),
// written in oracle/ref_driver's `ingest` output format so the tests compare it
// with the reference's own ingest byte for byte.
//   ingest_dev_main <mtx> <seed> <d> <out_prefix> [symmetric_input]
//   ingest_dev_main gen <path> <n> <m> <alpha> <seed>   (a Chung-Lu MatrixMarket file, written on all threads)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "nlp/ingest.hxx"
#include "nlp/predict.hxx"

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// endpoints i.i.d. with P(i) ~ i^-alpha (inverse CDF of the continuous law), self loops kept
static int gen(const char* path, uint64_t n, uint64_t m, double alpha, uint64_t seed) {
  const int T = 64;
  std::vector<std::string> parts(T);
#pragma omp parallel for schedule(static, 1)
  for (int t = 0; t < T; ++t) {
    const uint64_t a = m * t / T, b = m * (t + 1) / T;
    std::string& o = parts[t];
    o.reserve((b - a) * 18);
    char buf[48];
    const double e = 1.0 - alpha, N = std::pow((double)n, e);
    for (uint64_t i = a; i < b; ++i) {
      uint64_t id[2];
      for (int q = 0; q < 2; ++q) {
        const double x = (double)(mix(seed * 0x100000001B3ull ^ (2 * i + q)) >> 11) * (1.0 / 9007199254740992.0);
        uint64_t v = (uint64_t)std::pow(1.0 + x * (N - 1.0), 1.0 / e);
        id[q] = v < 1 ? 1 : (v > n ? n : v);
      }
      const int len = snprintf(buf, sizeof buf, "%llu %llu\n", (unsigned long long)id[0], (unsigned long long)id[1]);
      o.append(buf, len);
    }
  }
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  fprintf(f, "%%%%MatrixMarket matrix coordinate pattern general\n%llu %llu %llu\n", (unsigned long long)n,
          (unsigned long long)n, (unsigned long long)m);
  for (auto& p : parts) fwrite(p.data(), 1, p.size(), f);
  fclose(f);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 7 && std::string(argv[1]) == "gen")
    return gen(argv[2], strtoull(argv[3], nullptr, 10), strtoull(argv[4], nullptr, 10), atof(argv[5]),
               strtoull(argv[6], nullptr, 10));
  if (argc < 5) {
    fprintf(stderr, "usage: ingest_dev_main <mtx> <seed> <d> <out_prefix> [symmetric_input]\n");
    return 2;
  }
  uint32_t rng = (uint32_t)strtoul(argv[2], nullptr, 10);
  const double d = atof(argv[3]);
  const bool sym = argc > 5 && atoi(argv[5]) != 0;
  try {
    const double t0 = now_ms();
    nlp::MtxPairs mp = nlp::readMtxPairs(argv[1]);
    const double t1 = now_ms();
    nlp_dcsr* x = nullptr;
    nlp::check(nlp_dcsr_ingest(mp.src.empty() ? nullptr : mp.src.data(), mp.dst.empty() ? nullptr : mp.dst.data(),
                               mp.src.size(), mp.n, sym ? 1 : 0, 0, &x),
               "nlp_dcsr_ingest");
    const double t2 = now_ms();
    uint64_t span = 0, nnz = 0, rs = 0, ss = 0;
    nlp::check(nlp_dcsr_info(x, &span, &nnz, &rs, &ss), "nlp_dcsr_info");
    const uint64_t batch = (uint64_t)(d * nnz / 2);  // main.cxx:166
    std::vector<uint32_t> du(2 * batch + 1), dv(2 * batch + 1);
    uint64_t nd = 0;
    nlp_dcsr* y = nullptr;
    nlp::check(nlp_dcsr_delete_batch(x, batch, &rng, &y, du.data(), dv.data(), du.size(), &nd), "nlp_dcsr_delete_batch");
    const double t3 = now_ms();
    uint64_t S = 0, M = 0;
    nlp::check(nlp_dcsr_info(y, &S, &M, nullptr, nullptr), "nlp_dcsr_info");
    std::vector<uint64_t> off(S + 1);
    std::vector<uint32_t> keys(M);
    nlp::check(nlp_dcsr_copy(y, off.data(), keys.data()), "nlp_dcsr_copy");
    const std::string out = argv[4];
    FILE* f = fopen((out + ".csr").c_str(), "wb");
    if (!f) return 1;
    fwrite(&S, 8, 1, f);
    fwrite(&M, 8, 1, f);
    fwrite(off.data(), 8, off.size(), f);
    if (M) fwrite(keys.data(), 4, M, f);
    fclose(f);
    f = fopen((out + ".del").c_str(), "wb");
    if (!f) return 1;
    fwrite(&nd, 8, 1, f);
    for (uint64_t i = 0; i < nd; ++i) {
      fwrite(&du[i], 4, 1, f);
      fwrite(&dv[i], 4, 1, f);
    }
    fclose(f);
    printf("{\"order\": %llu, \"size\": %llu, \"read_size\": %llu, \"symmetrize_size\": %llu, \"deletions\": %llu, "
           "\"lines\": %zu, \"parse_ms\": %.1f, \"ingest_ms\": %.1f, \"delete_ms\": %.1f}\n",
           (unsigned long long)(span - 1), (unsigned long long)nnz, (unsigned long long)rs, (unsigned long long)ss,
           (unsigned long long)nd, mp.src.size(), t1 - t0, t2 - t1, t3 - t2);
    nlp_dcsr_destroy(y);
    nlp_dcsr_destroy(x);
  } catch (const std::exception& e) {
    fprintf(stderr, "ingest_dev_main: %s\n", e.what());
    return 1;
  }
  return 0;
}
