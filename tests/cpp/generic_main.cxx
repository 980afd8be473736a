// Generic entry points of include/nlp/predict.hxx with user score lambdas
// (predictLinksWithIntersectionBasic[Omp], predictLinksWithIntersection[Omp]
// with CUSTOMVALUE = false, predict.hxx:358-490).
//   generic_main <csr> <H> <maxEdges> <out_prefix>
// writes <out_prefix>.jac_generic / .jac_builtin (the reference's own Jaccard
// lambda, predict.hxx:557-559, through the generic entry vs the built-in
// metric) and .custom (a count-based lambda the test recomputes on the host).
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <vector>
#include "nlp/predict.hxx"

struct CsrGraph {
  using key_type = uint32_t;
  std::vector<uint64_t> off;
  std::vector<uint32_t> keys;
  size_t span() const { return off.size() - 1; }
  bool hasVertex(uint32_t u) const { return u < span(); }
  size_t degree(uint32_t u) const { return u < span() ? size_t(off[u + 1] - off[u]) : 0; }
  template <class F> void forEachEdgeKey(uint32_t u, F f) const {
    for (uint64_t i = off[u]; i < off[u + 1]; ++i) f(keys[i]);
  }
};

template <class R>
static void dump(const R& r, const std::string& path) {
  FILE* f = fopen(path.c_str(), "wb");
  uint64_t n = r.edges.size();
  fwrite(&n, 8, 1, f);
  for (auto& [u, v, s] : r.edges) { fwrite(&u, 4, 1, f); fwrite(&v, 4, 1, f); float x = float(s); fwrite(&x, 4, 1, f); }
  fclose(f);
}

template <int H>
static int run(const CsrGraph& x, size_t k, const std::string& pre) {
  using W = float;
  auto jac = [&](auto u, auto v, auto Nuv) { return W(Nuv) / (x.degree(u) + x.degree(v) - Nuv); };
  auto a = predictLinksWithIntersectionBasicOmp<H>(x, PredictLinkOptions<W>(1, k), jac);
  auto b = predictLinksJaccardCoefficientOmp<H>(x, PredictLinkOptions<W>(1, k));
  auto fu = [](auto& e, auto u, auto v) { ++e; };
  auto custom = [](auto u, auto v, auto Nuv) { return W(Nuv) * 0.5f + 1.0f / W(u % 7 + 1); };
  auto c = predictLinksWithIntersectionOmp<H, 0, false, false>(x, PredictLinkOptions<W>(1, k), uint32_t(), custom, fu);
  dump(a, pre + ".jac_generic");
  dump(b, pre + ".jac_builtin");
  dump(c, pre + ".custom");
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  uint64_t S, M;
  if (fread(&S, 8, 1, f) != 1 || fread(&M, 8, 1, f) != 1) return 2;
  CsrGraph g;
  g.off.resize(S + 1);
  g.keys.resize(M);
  if (fread(g.off.data(), 8, S + 1, f) != S + 1 || (M && fread(g.keys.data(), 4, M, f) != M)) return 2;
  fclose(f);
  const int H = atoi(argv[2]);
  const size_t k = size_t(atoll(argv[3]));
  try {
    switch (H) {
      case 0: return run<0>(g, k, argv[4]);
      case 4: return run<4>(g, k, argv[4]);
      case 8: return run<8>(g, k, argv[4]);
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 3;
  }
  return 2;
}
