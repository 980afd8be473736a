// C++ drop-in check: a main.cxx-style caller of include/nlp/predict.hxx.
// Reads a CSR (oracle/pyoracle.py write_csr format), runs every metric through
// the reference's template names on (a) a graph-concept type and (b) a resident
// nlp::HipGraph, and writes the edges of (b) for comparison with the oracle.
//   predict_main <csr> <H> <maxEdges> <out_prefix>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <string>
#include "nlp/predict.hxx"

// Minimal graph concept (Graph.hxx:59-169): key_type, span, hasVertex, forEachEdgeKey.
struct CsrGraph {
  using key_type = uint32_t;
  std::vector<uint64_t> off;
  std::vector<uint32_t> keys;
  size_t span() const { return off.size() - 1; }
  bool hasVertex(uint32_t u) const { return u < span(); }
  template <class F> void forEachEdgeKey(uint32_t u, F f) const {
    for (uint64_t i = off[u]; i < off[u + 1]; ++i) f(keys[i]);
  }
};

template <class R>
static void dump(const R& r, const std::string& path) {
  FILE* f = fopen(path.c_str(), "wb");
  uint64_t n = r.edges.size();
  fwrite(&n, 8, 1, f);
  for (auto& [u, v, s] : r.edges) { fwrite(&u, 4, 1, f); fwrite(&v, 4, 1, f); fwrite(&s, 4, 1, f); }
  fclose(f);
}

#define RUN(NAME, IDX)                                                                   \
  {                                                                                      \
    auto a = predictLinks##NAME##Omp<HUB>(g, PredictLinkOptions<float>(1, k));          \
    auto b = predictLinks##NAME##Hip<HUB>(hg, PredictLinkOptions<float>(1, k));         \
    auto c = predictLinks##NAME<HUB>(hg, PredictLinkOptions<float>(1, k));              \
    if (a.edges != b.edges || b.edges != c.edges) { fprintf(stderr, #NAME " mismatch\n"); return 1; } \
    dump(b, prefix + "." + std::to_string(IDX));                                         \
  }

template <int HUB>
static int run(const CsrGraph& g, size_t k, const std::string& prefix) {
  nlp::HipGraph hg(g);
  RUN(CommonNeighbors, 0) RUN(JaccardCoefficient, 1) RUN(SorensenIndex, 2) RUN(SaltonCosineSimilarity, 3)
  RUN(HubPromoted, 4) RUN(HubDepressed, 5) RUN(LeichtHolmeNermanScore, 6) RUN(AdamicAdarCoefficient, 7)
  RUN(ResourceAllocationScore, 8)
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
  int H = atoi(argv[2]);
  size_t k = size_t(atoll(argv[3]));
  std::string prefix = argv[4];
  try {
    switch (H) {
      case 0: return run<0>(g, k, prefix);
      case 4: return run<4>(g, k, prefix);
      case 8: return run<8>(g, k, prefix);
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 3;
  }
  return 2;
}
