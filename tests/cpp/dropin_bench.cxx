// The drop-in header's cost per call, as main.cxx pays it:
// predictLinksJaccardCoefficientOmp<H>(x, {1, k}) through include/nlp/predict.hxx
// on a host graph -- the fingerprint of the graph (the resident copy is reused
// across calls, detail::cachedGraph), the prediction, the copy of the k links
// to the host and the vector<tuple> the reference returns (main.cxx:50).
// The graph is a DiGraphCsr-shaped struct (offsets / degrees / edgeKeys,
// Graph.hxx:396-406) read from the CSR file bench.py writes for the reference
// driver.  Prints one JSON object.
//   dropin_bench <csr> <k> <H,H,...> [calls per H]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "nlp/predict.hxx"

struct CsrView {  // the DiGraphCsr members the header reads directly
  using key_type = uint32_t;
  std::vector<uint64_t> offsets;
  std::vector<uint32_t> degrees;
  std::vector<uint32_t> edgeKeys;
  size_t span() const { return degrees.size(); }
  bool hasVertex(uint32_t u) const { return u < span(); }
};

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int H>
static void run(const CsrView& g, const nlp::HipGraph& gh, size_t k, int calls, std::string& js) {
  double first = 0, sum = 0, lib = 0, hsum = 0, hlib = 0;
  size_t n = 0;
  for (int i = 0; i <= calls; ++i) {
    const double t0 = now_ms();
    auto r = predictLinksJaccardCoefficientOmp<H>(g, PredictLinkOptions<float>(1, k));
    const double t = now_ms() - t0;
    if (i == 0) {
      first = t;
    } else {
      sum += t;
      lib += r.time;
    }
    n = r.edges.size();
  }
  // route (b) of INTEGRATION.md: the same call on a resident nlp::HipGraph (no content check per call)
  for (int i = 0; i <= calls; ++i) {
    const double t0 = now_ms();
    auto r = predictLinksJaccardCoefficientOmp<H>(gh, PredictLinkOptions<float>(1, k));
    const double t = now_ms() - t0;
    if (i > 0) {
      hsum += t;
      hlib += r.time;
    }
    if (r.edges.size() != n) n = size_t(-1);  // the two routes must agree
  }
  char b[768];
  snprintf(b, sizeof b, "%s{\"H\": %d, \"first_call_ms\": %.3f, \"dropin_ms_per_call\": %.3f, \"library_ms_per_call\": %.3f, "
           "\"overhead_ms_per_call\": %.3f, \"handle_ms_per_call\": %.3f, \"handle_overhead_ms_per_call\": %.3f, "
           "\"predicted\": %zu, \"calls\": %d}",
           js.empty() ? "" : ", ", H, first, sum / calls, lib / calls, (sum - lib) / calls, hsum / calls,
           (hsum - hlib) / calls, n, calls);
  js += b;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: dropin_bench <csr> <k> <H,H,...> [calls]\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  uint64_t hdr[2];
  if (fread(hdr, 8, 2, f) != 2) return 2;
  CsrView g;
  std::vector<uint64_t> off(hdr[0] + 1);
  g.edgeKeys.resize(hdr[1]);
  if (fread(off.data(), 8, off.size(), f) != off.size()) return 2;
  if (fread(g.edgeKeys.data(), 4, g.edgeKeys.size(), f) != g.edgeKeys.size()) return 2;
  fclose(f);
  g.offsets = off;
  g.degrees.resize(hdr[0]);
  for (uint64_t u = 0; u < hdr[0]; ++u) g.degrees[u] = uint32_t(off[u + 1] - off[u]);
  const size_t k = strtoull(argv[2], nullptr, 10);
  const int calls = argc > 4 ? atoi(argv[4]) : 3;
  std::string js;
  uint64_t m = 0;
  const double f0 = now_ms();
  (void)nlp::graphFingerprint(g, &m);
  const double fp = now_ms() - f0;
  const double u0 = now_ms();
  const nlp::HipGraph& gh = nlp::detail::cachedGraph(g);  // the resident copy (fingerprint, CSR, upload, per-graph build)
  const double upload = now_ms() - u0;
  for (const char* p = argv[3]; *p;) {
    const int h = atoi(p);
    if (h == 4) run<4>(g, gh, k, calls, js);
    else if (h == 8) run<8>(g, gh, k, calls, js);
    else if (h == 16) run<16>(g, gh, k, calls, js);
    else if (h == 32) run<32>(g, gh, k, calls, js);
    while (*p && *p != ',') ++p;
    if (*p) ++p;
  }
  printf("{\"fingerprint_ms\": %.3f, \"entries\": %llu, \"first_upload_ms\": %.3f, \"calls\": [%s]}\n", fp,
         (unsigned long long)m, upload, js.c_str());
  return 0;
}
