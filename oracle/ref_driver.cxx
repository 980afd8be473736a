// ref_driver.cxx -- our own driver around the REAL reference headers.
//
// TEST INFRASTRUCTURE ONLY (oracle).  Compiled by oracle/Makefile against
// /root/reference/inc/main.hxx where it lies (nothing is copied); the binary
// lands in oracle/_ref/ (git-ignored, travels to the GPU box as a build
// product).  It is used to:
//   * generate the golden fixtures in tests/golden/ (make_golden.py), and
//   * time the reference's own OpenMP path as bench.py's cpu_baseline
//     (kind "reference").
//
// Modes
//   ingest  <mtx> <seed> <d> <out_prefix>
//       readMtxOmpW -> symmetrizeOmp -> removeSelfLoopsOmpU   (main.cxx:241-245)
//       y = duplicate(x); generateEdgeDeletions(rnd(seed), y, d*|E|/2, 1, span-1, true);
//       tidyBatchUpdateU; applyBatchUpdateOmpU                  (main.cxx:164-169)
//       writes <out_prefix>.csr  (u64 span, u64 M, u64 off[span+1], u32 keys[M])
//              <out_prefix>.del  (u64 n, u32 pairs[2n])  directed, sorted, unique
//   predict <csr> <metric 0..8> <H> <maxEdges|-1> <seq|omp> <threads> <repeat> <out> [maxfactor2]
//       runs predictLinks<Metric>[Omp]<H, MAXFACTOR2>(G, {repeat, maxEdges}) on a
//       DiGraphCsr built from <csr>; writes u64 n, then n x {u32 u, u32 w, f32 score};
//       prints "time_ms scoring_ms n" on stdout.  MAXFACTOR2 in {0, 1, 2, 4}
//       (non-zero only with H in {0, 4}).
//   time    <csr> <metric> <H> <maxEdges> <threads> <repeat>
//       same as predict/omp without writing the edges (CPU baseline).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>
#include <tuple>
#include <random>
#include <stdexcept>
#include "/root/reference/inc/main.hxx"

using namespace std;
using K = uint32_t;
using Csr = DiGraphCsr<K, None, None, size_t>;

static void die(const char* m) { fprintf(stderr, "ref_driver: %s\n", m); exit(2); }

static void writeCsr(const string& path, const vector<uint64_t>& off, const vector<K>& keys) {
  FILE* f = fopen(path.c_str(), "wb"); if (!f) die("cannot write csr");
  uint64_t S = off.size() - 1, M = keys.size();
  fwrite(&S, 8, 1, f); fwrite(&M, 8, 1, f);
  fwrite(off.data(), 8, off.size(), f);
  if (M) fwrite(keys.data(), 4, M, f);
  fclose(f);
}

static Csr readCsr(const string& path) {
  FILE* f = fopen(path.c_str(), "rb"); if (!f) die("cannot read csr");
  uint64_t S, M;
  if (fread(&S, 8, 1, f) != 1 || fread(&M, 8, 1, f) != 1) die("bad csr header");
  Csr g(S, M);
  vector<uint64_t> off(S + 1);
  if (fread(off.data(), 8, S + 1, f) != S + 1) die("bad csr offsets");
  if (M && fread(g.edgeKeys.data(), 4, M, f) != M) die("bad csr keys");
  fclose(f);
  for (uint64_t u = 0; u <= S; ++u) g.offsets[u] = off[u];
  for (uint64_t u = 0; u < S; ++u) g.degrees[u] = K(off[u + 1] - off[u]);
  return g;
}

static int doIngest(int argc, char** argv) {
  if (argc < 6) die("ingest <mtx> <seed> <d> <out_prefix>");
  const char* mtx = argv[2];
  unsigned seed = unsigned(strtoul(argv[3], nullptr, 10));
  double d = atof(argv[4]);
  string out = argv[5];
  DiGraph<K, None, float> x;
  readMtxOmpW(x, mtx, false);
  x = symmetrizeOmp(x);
  auto fl = [](auto u) { return true; };
  removeSelfLoopsOmpU(x, fl);
  default_random_engine rnd(seed);
  auto y = duplicate(x);
  auto del = generateEdgeDeletions(rnd, y, size_t(d * x.size() / 2), 1, x.span() - 1, true);
  vector<tuple<K, K>> ins;
  tidyBatchUpdateU(del, ins, y);
  applyBatchUpdateOmpU(y, del, ins);
  vector<uint64_t> off(y.span() + 1, 0);
  vector<K> keys; keys.reserve(y.size());
  for (K u = 0; u < y.span(); ++u) {
    off[u] = keys.size();
    y.forEachEdgeKey(u, [&](auto v) { keys.push_back(v); });
  }
  off[y.span()] = keys.size();
  writeCsr(out + ".csr", off, keys);
  FILE* f = fopen((out + ".del").c_str(), "wb"); if (!f) die("cannot write del");
  uint64_t n = del.size();
  fwrite(&n, 8, 1, f);
  for (auto& [u, v] : del) { fwrite(&u, 4, 1, f); fwrite(&v, 4, 1, f); }
  fclose(f);
  printf("order %zu size %zu span %zu deletions %zu (x: order %zu size %zu)\n",
         y.order(), y.size(), y.span(), del.size(), x.order(), x.size());
  return 0;
}

template <int H, bool OMP, int F = 0>
static PredictLinkResult<K, float> runMetric(const Csr& g, int metric, const PredictLinkOptions<float>& o) {
  switch (metric) {
    case 0: return OMP ? predictLinksCommonNeighborsOmp<H, F>(g, o)         : predictLinksCommonNeighbors<H, F>(g, o);
    case 1: return OMP ? predictLinksJaccardCoefficientOmp<H, F>(g, o)      : predictLinksJaccardCoefficient<H, F>(g, o);
    case 2: return OMP ? predictLinksSorensenIndexOmp<H, F>(g, o)           : predictLinksSorensenIndex<H, F>(g, o);
    case 3: return OMP ? predictLinksSaltonCosineSimilarityOmp<H, F>(g, o)  : predictLinksSaltonCosineSimilarity<H, F>(g, o);
    case 4: return OMP ? predictLinksHubPromotedOmp<H, F>(g, o)             : predictLinksHubPromoted<H, F>(g, o);
    case 5: return OMP ? predictLinksHubDepressedOmp<H, F>(g, o)            : predictLinksHubDepressed<H, F>(g, o);
    case 6: return OMP ? predictLinksLeichtHolmeNermanScoreOmp<H, F>(g, o)  : predictLinksLeichtHolmeNermanScore<H, F>(g, o);
    case 7: return OMP ? predictLinksAdamicAdarCoefficientOmp<H, F>(g, o)   : predictLinksAdamicAdarCoefficient<H, F>(g, o);
    case 8: return OMP ? predictLinksResourceAllocationScoreOmp<H, F>(g, o) : predictLinksResourceAllocationScore<H, F>(g, o);
  }
  die("bad metric");
  return {};
}

template <bool OMP, int F>
static PredictLinkResult<K, float> dispatchF(const Csr& g, int metric, int H, const PredictLinkOptions<float>& o) {
  switch (H) {
    case 0: return runMetric<0, OMP, F>(g, metric, o);
    case 4: return runMetric<4, OMP, F>(g, metric, o);
  }
  die("MAXFACTOR2 needs H in {0, 4}");
  return {};
}

template <bool OMP>
static PredictLinkResult<K, float> dispatch(const Csr& g, int metric, int H, const PredictLinkOptions<float>& o,
                                            int F) {
  switch (F) {
    case 0: break;
    case 1: return dispatchF<OMP, 1>(g, metric, H, o);
    case 2: return dispatchF<OMP, 2>(g, metric, H, o);
    case 4: return dispatchF<OMP, 4>(g, metric, H, o);
    default: die("unsupported MAXFACTOR2");
  }
  switch (H) {  // the MINDEGREE1 sweep of main.cxx:67-80, plus 1 and 3 for edge cases
    case 0:    return runMetric<0, OMP>(g, metric, o);
    case 1:    return runMetric<1, OMP>(g, metric, o);
    case 2:    return runMetric<2, OMP>(g, metric, o);
    case 3:    return runMetric<3, OMP>(g, metric, o);
    case 4:    return runMetric<4, OMP>(g, metric, o);
    case 8:    return runMetric<8, OMP>(g, metric, o);
    case 16:   return runMetric<16, OMP>(g, metric, o);
    case 32:   return runMetric<32, OMP>(g, metric, o);
    case 64:   return runMetric<64, OMP>(g, metric, o);
    case 128:  return runMetric<128, OMP>(g, metric, o);
    case 256:  return runMetric<256, OMP>(g, metric, o);
    case 512:  return runMetric<512, OMP>(g, metric, o);
    case 1024: return runMetric<1024, OMP>(g, metric, o);
  }
  die("unsupported H");
  return {};
}

static int doPredict(int argc, char** argv, bool write) {
  // predict <csr> <metric> <H> <maxEdges> <seq|omp> <threads> <repeat> <out>
  // time    <csr> <metric> <H> <maxEdges> <threads> <repeat>
  int need = write ? 10 : 8;
  if (argc < need) die("bad args");
  Csr g = readCsr(argv[2]);
  int metric = atoi(argv[3]);
  int H = atoi(argv[4]);
  long long me = atoll(argv[5]);
  size_t maxEdges = me < 0 ? size_t(-1) : size_t(me);
  bool omp = write ? string(argv[6]) == "omp" : true;
  int threads = atoi(argv[write ? 7 : 6]);
  int repeat = atoi(argv[write ? 8 : 7]);
  const int F = write && argc > 10 ? atoi(argv[10]) : 0;
  omp_set_num_threads(threads);
  PredictLinkOptions<float> o(repeat, maxEdges);
  auto r = omp ? dispatch<true>(g, metric, H, o, F) : dispatch<false>(g, metric, H, o, F);
  printf("%.3f %.3f %zu\n", r.time, r.scoringTime, r.edges.size());
  if (write) {
    FILE* f = fopen(argv[9], "wb"); if (!f) die("cannot write out");
    uint64_t n = r.edges.size();
    fwrite(&n, 8, 1, f);
    // packed {u, w, score} records, written in blocks (a full-size top-k is 1e8+ links)
    vector<uint32_t> buf;
    const size_t blk = size_t(1) << 22;
    for (size_t i = 0; i < n; i += blk) {
      const size_t e = std::min(n, i + blk);
      buf.resize(3 * (e - i));
      for (size_t j = i; j < e; ++j) {
        auto& [u, v, s] = r.edges[j];
        buf[3 * (j - i)] = u;
        buf[3 * (j - i) + 1] = v;
        memcpy(&buf[3 * (j - i) + 2], &s, 4);
      }
      if (fwrite(buf.data(), 4, buf.size(), f) != buf.size()) die("short write");
    }
    fclose(f);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) die("mode: ingest | predict | time");
  string mode = argv[1];
  if (mode == "ingest") return doIngest(argc, argv);
  if (mode == "predict") return doPredict(argc, argv, true);
  if (mode == "time") return doPredict(argc, argv, false);
  die("unknown mode");
  return 1;
}
