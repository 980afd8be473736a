// nlp/predict.hxx -- drop-in C++ API of the reference's predict.hxx, backed by
// the MI355X library (libnlp.so, include/nlp.h).
//
// Reference: /root/reference/inc/predict.hxx.  main.cxx calls
//     auto p1 = predictLinksJaccardCoefficientOmp<deg>(y, {repeat, k});   (main.cxx:50)
// With this header instead of the reference's, the same line runs on the GPU.
// Provided, with the reference's template signatures
//     template <int MINDEGREE1=4, int MAXFACTOR2=0, bool FORCEHEAP=false, class G, class W=float>
//     auto f(const G& x, const PredictLinkOptions<W>& o={}) -> PredictLinkResult<typename G::key_type, W>
// for the nine metrics, each as predictLinks<Metric>, predictLinks<Metric>Omp
// and predictLinks<Metric>Hip (all three run the HIP path; the reference's
// sequential / OpenMP split is a CPU scheduling detail):
//     CommonNeighbors, JaccardCoefficient, SorensenIndex, SaltonCosineSimilarity,
//     HubPromoted, HubDepressed, LeichtHolmeNermanScore, AdamicAdarCoefficient,
//     ResourceAllocationScore                                  (predict.hxx:502-831)
//
// Differences from the reference (all documented in DESIGN.md):
//   * results are deterministic: ties at the k-th score are filled in
//     (u asc, v asc) order; the reference's tie choice depends on the OpenMP
//     schedule;
//   * with fewer candidates than maxEdges all candidates are returned (the
//     reference's OpenMP merge reads out of bounds, A.2);
//   * MAXFACTOR2 > 0 keeps a candidate w of u only when deg(w) <= MAXFACTOR2 *
//     deg(u), the reference's second-hop filter (predict.hxx:221,295; its other
//     clause, deg(u) <= MAXFACTOR2 * deg(u), always holds); FORCEHEAP only
//     changes the reference's heap bookkeeping and is accepted and ignored;
//   * the generic predictLinksWithIntersection[Omp](x, o, VT, fs, fu) takes
//     arbitrary lambdas, which cannot cross the C ABI: not provided;
//   * errors throw std::runtime_error (the reference has no error reporting).
//
// Graph input: any type with the reference's graph concept (Graph.hxx):
// key_type, span(), hasVertex(u), forEachEdgeKey(u, fn) -- DiGraph and
// DiGraphCsr both qualify.  It is converted to a CSR with identity vertex ids
// (absent vertices get empty rows) and uploaded on every call; keep a
// nlp::HipGraph to upload once and call many times (main.cxx runs 99
// predictions per graph).
#pragma once
#include <cstdint>
#include <cstddef>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../nlp.h"

#pragma region TYPES
/** Options for Link Prediction algorithm (predict.hxx:33-55). */
template <class W>
struct PredictLinkOptions {
  /** Number of times to repeat the algorithm [1]. */
  int repeat;
  /** Maximum number of edges to predict [-1]. */
  size_t maxEdges;
  /** Minimum score above which to consider a link [0]. */
  W minScore;
  PredictLinkOptions(int repeat = 1, size_t maxEdges = size_t(-1), W minScore = W())
      : repeat(repeat), maxEdges(maxEdges), minScore(minScore) {}
};

/** Result of Link Prediction algorithm (predict.hxx:65-102). */
template <class K, class W>
struct PredictLinkResult {
  /** Predicted links (undirected), score descending. */
  std::vector<std::tuple<K, K, W>> edges;
  /** Total time spent in milliseconds. */
  float time;
  /** Time spent in milliseconds for scoring. */
  float scoringTime;
  PredictLinkResult() : edges(), time(), scoringTime() {}
  PredictLinkResult(std::vector<std::tuple<K, K, W>>&& edges, float time = 0, float scoringTime = 0)
      : edges(std::move(edges)), time(time), scoringTime(scoringTime) {}
};
#pragma endregion

namespace nlp {

inline void check(nlp_status s, const char* what) {
  if (s != NLP_OK) throw std::runtime_error(std::string(what) + ": " + nlp_status_string(s));
}

/** Build the identity-id CSR of any graph concept G (csr.hxx:106-222 layout,
 *  without the dense renumbering so vertex ids are preserved). */
template <class G>
inline void graphToCsr(const G& x, std::vector<uint64_t>& offsets, std::vector<uint32_t>& keys) {
  const size_t S = x.span();
  offsets.assign(S + 1, 0);
  keys.clear();
  for (size_t u = 0; u < S; ++u) {
    offsets[u] = keys.size();
    if (!x.hasVertex(typename G::key_type(u))) continue;
    x.forEachEdgeKey(typename G::key_type(u), [&](auto v) { keys.push_back(uint32_t(v)); });
  }
  offsets[S] = keys.size();
}

/** A graph resident in HBM (one nlp_graph handle). */
class HipGraph {
 public:
  using key_type = uint32_t;
  HipGraph() = default;
  HipGraph(const uint64_t* offsets, const uint32_t* keys, uint64_t span, int device = 0) {
    check(nlp_graph_create(offsets, keys, span, device, &g_), "nlp_graph_create");
  }
  template <class G>
  explicit HipGraph(const G& x, int device = 0) {
    std::vector<uint64_t> off;
    std::vector<uint32_t> keys;
    graphToCsr(x, off, keys);
    check(nlp_graph_create(off.data(), keys.empty() ? nullptr : keys.data(), off.size() - 1, device, &g_),
          "nlp_graph_create");
  }
  HipGraph(const HipGraph&) = delete;
  HipGraph& operator=(const HipGraph&) = delete;
  HipGraph(HipGraph&& o) noexcept : g_(o.g_) { o.g_ = nullptr; }
  HipGraph& operator=(HipGraph&& o) noexcept {
    if (this != &o) { reset(); g_ = o.g_; o.g_ = nullptr; }
    return *this;
  }
  ~HipGraph() { reset(); }
  void reset() {
    if (g_) nlp_graph_destroy(g_);
    g_ = nullptr;
  }
  nlp_graph* get() const { return g_; }
  size_t span() const {
    uint64_t s = 0;
    nlp_graph_info(g_, &s, nullptr, nullptr, nullptr);
    return size_t(s);
  }

 private:
  nlp_graph* g_ = nullptr;
};

/** predictLinks<Metric>Omp on a resident graph. */
template <class K = uint32_t, class W = float>
inline PredictLinkResult<K, W> predictLinksHip(const HipGraph& g, nlp_metric metric, uint32_t mindegree1,
                                               const PredictLinkOptions<W>& o, uint32_t maxfactor2 = 0) {
  nlp_timing t{};
  uint64_t n = 0;
  const uint64_t me = o.maxEdges == size_t(-1) ? UINT64_MAX : uint64_t(o.maxEdges);
  std::vector<nlp_edge> buf;
  if (me == UINT64_MAX) {  // all candidates: predict once (count query), then fetch the kept result
    check(nlp_predict_ex(g.get(), metric, mindegree1, maxfactor2, float(o.minScore), me, o.repeat, nullptr, &n, &t),
          "nlp_predict_ex");
    buf.resize(n);
    uint64_t got = 0;
    check(nlp_copy_last(g.get(), buf.data(), n, &got), "nlp_copy_last");
    n = got;
  } else {
    buf.resize(me);
    check(nlp_predict_ex(g.get(), metric, mindegree1, maxfactor2, float(o.minScore), me, o.repeat,
                         me ? buf.data() : nullptr, &n, &t),
          "nlp_predict_ex");
  }
  std::vector<std::tuple<K, K, W>> a;
  a.reserve(n);
  for (uint64_t i = 0; i < n; ++i) a.emplace_back(K(buf[i].u), K(buf[i].v), W(buf[i].score));
  return PredictLinkResult<K, W>(std::move(a), t.total_ms, t.score_ms);
}

template <class G, class W>
inline PredictLinkResult<typename G::key_type, W> predictLinksHipAny(const G& x, nlp_metric metric,
                                                                     uint32_t mindegree1,
                                                                     const PredictLinkOptions<W>& o,
                                                                     uint32_t maxfactor2 = 0) {
  HipGraph g(x);
  return predictLinksHip<typename G::key_type, W>(g, metric, mindegree1, o, maxfactor2);
}

template <class W>
inline PredictLinkResult<uint32_t, W> predictLinksHipAny(const HipGraph& g, nlp_metric metric, uint32_t mindegree1,
                                                         const PredictLinkOptions<W>& o, uint32_t maxfactor2 = 0) {
  return predictLinksHip<uint32_t, W>(g, metric, mindegree1, o, maxfactor2);
}

}  // namespace nlp

// The 27 entry points: predictLinks<Metric>, predictLinks<Metric>Omp, predictLinks<Metric>Hip.
#define NLP_DEFINE_PREDICTOR(NAME, METRIC)                                                                 \
  template <int MINDEGREE1 = 4, int MAXFACTOR2 = 0, bool FORCEHEAP = false, class G, class W = float>    \
  inline auto predictLinks##NAME(const G& x, const PredictLinkOptions<W>& o = {}) {                      \
    static_assert(MINDEGREE1 >= 0 && MAXFACTOR2 >= 0, "negative MINDEGREE1 / MAXFACTOR2");              \
    return nlp::predictLinksHipAny(x, METRIC, uint32_t(MINDEGREE1), o, uint32_t(MAXFACTOR2));           \
  }                                                                                                       \
  template <int MINDEGREE1 = 4, int MAXFACTOR2 = 0, bool FORCEHEAP = false, class G, class W = float>    \
  inline auto predictLinks##NAME##Omp(const G& x, const PredictLinkOptions<W>& o = {}) {                 \
    static_assert(MINDEGREE1 >= 0 && MAXFACTOR2 >= 0, "negative MINDEGREE1 / MAXFACTOR2");              \
    return nlp::predictLinksHipAny(x, METRIC, uint32_t(MINDEGREE1), o, uint32_t(MAXFACTOR2));           \
  }                                                                                                       \
  template <int MINDEGREE1 = 4, int MAXFACTOR2 = 0, bool FORCEHEAP = false, class G, class W = float>    \
  inline auto predictLinks##NAME##Hip(const G& x, const PredictLinkOptions<W>& o = {}) {                 \
    static_assert(MINDEGREE1 >= 0 && MAXFACTOR2 >= 0, "negative MINDEGREE1 / MAXFACTOR2");              \
    return nlp::predictLinksHipAny(x, METRIC, uint32_t(MINDEGREE1), o, uint32_t(MAXFACTOR2));           \
  }

NLP_DEFINE_PREDICTOR(CommonNeighbors, NLP_CN)
NLP_DEFINE_PREDICTOR(JaccardCoefficient, NLP_JAC)
NLP_DEFINE_PREDICTOR(SorensenIndex, NLP_SOR)
NLP_DEFINE_PREDICTOR(SaltonCosineSimilarity, NLP_SAL)
NLP_DEFINE_PREDICTOR(HubPromoted, NLP_HPI)
NLP_DEFINE_PREDICTOR(HubDepressed, NLP_HDI)
NLP_DEFINE_PREDICTOR(LeichtHolmeNermanScore, NLP_LHN)
NLP_DEFINE_PREDICTOR(AdamicAdarCoefficient, NLP_AA)
NLP_DEFINE_PREDICTOR(ResourceAllocationScore, NLP_RA)
#undef NLP_DEFINE_PREDICTOR
