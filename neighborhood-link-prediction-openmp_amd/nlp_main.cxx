// nlp_main.cxx -- the reference experiment driver (main.cxx) on the MI355X
// library: SURVEY.md §8(f) N4, with N1/N2 on the device (the MatrixMarket
// pairs parsed on all host threads by nlp::readMtxPairs, then nlp_dcsr_ingest
// and nlp_dcsr_delete_batch; NLP_HOST_INGEST=1: the host restatement
// nlp/ingest.hxx) and the N3 device evaluation (nlp_set_truth / nlp_last_common).
//
//   nlp_main <graph.mtx> [symmetric=0] [weighted=0]
//
// Same flow and log lines as main.cxx:190-249 (parsed by the reference's
// process.js): load, symmetrize unless the input is symmetric, remove
// self-loops, then for every deletion batch (runBatches, main.cxx:157-179)
// predict with the nine metrics x eleven hub thresholds (PREDICT_LINKS_ALL,
// main.cxx:67-80; maxEdges = |deletions0| / 2, main.cxx:50) and print
//   {-0.000e+00/+<d> batchf, <T> threads} -> {<time>ms, <scoring>ms scoring,
//    <precision> precision, <recall> recall} predictLinks<Metric>Hip<H>
// Configuration by environment, with main.sh's names and defaults:
//   BATCH_DELETIONS_BEGIN=0.0001 BATCH_DELETIONS_END=0.1 BATCH_DELETIONS_STEP=*=10
//   REPEAT_BATCH=1 BATCH_LENGTH=1 REPEAT_METHOD=1 MAX_THREADS (printed only)
// and NLP_SEED (default: std::random_device, like main.cxx:194-195),
// NLP_DEVICE=0, NLP_METRICS=CN,JAC,... (default all), NLP_HUBS=0,2,...,1024.
// Weighted input is read as a pattern (the scores never use edge weights).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "nlp/ingest.hxx"
#include "nlp/predict.hxx"

namespace {

double envd(const char* k, double def) {
  const char* v = getenv(k);
  return v && *v ? atof(v) : def;
}
int envi(const char* k, int def) {
  const char* v = getenv(k);
  return v && *v ? atoi(v) : def;
}
std::vector<std::string> envlist(const char* k, const char* def) {
  const char* v = getenv(k);
  std::stringstream ss(v && *v ? v : def);
  std::vector<std::string> out;
  std::string x;
  while (std::getline(ss, x, ',')) out.push_back(x);
  return out;
}

// BATCH_*_STEP: "*=10" or "+=0.01" (main.sh:24, main.cxx:174)
double step(double d, const char* spec) {
  if (!spec || strlen(spec) < 3) return d * 10;
  const double a = atof(spec + 2);
  return spec[0] == '*' ? d * a : d + a;
}

void printGraph(const nlp::HostCsr& x, const char* suffix) {  // writeGraphSizes (Graph.hxx:653-657)
  printf("order: %zu size: %zu [directed] {}%s\n", x.span() ? x.span() - 1 : 0, x.size(), suffix);
}

struct Metric {
  const char* name;   // enum name (nlp.h)
  const char* func;   // predict.hxx function name
  nlp_metric id;
};
const Metric METRICS[] = {
    {"CN", "predictLinksCommonNeighborsHip", NLP_CN},
    {"JAC", "predictLinksJaccardCoefficientHip", NLP_JAC},
    {"SOR", "predictLinksSorensenIndexHip", NLP_SOR},
    {"SAL", "predictLinksSaltonCosineSimilarityHip", NLP_SAL},
    {"HPI", "predictLinksHubPromotedHip", NLP_HPI},
    {"HDI", "predictLinksHubDepressedHip", NLP_HDI},
    {"LHN", "predictLinksLeichtHolmeNermanScoreHip", NLP_LHN},
    {"AA", "predictLinksAdamicAdarCoefficientHip", NLP_AA},
    {"RA", "predictLinksResourceAllocationScoreHip", NLP_RA},
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: nlp_main <graph.mtx> [symmetric=0] [weighted=0]\n");
    return 2;
  }
  const char* file = argv[1];
  const bool symmetric = argc > 2 && atoi(argv[2]) != 0;
  const int threads = envi("MAX_THREADS", 1);
  const int repeat = envi("REPEAT_METHOD", 1), repeatBatch = envi("REPEAT_BATCH", 1);
  const int batchLength = envi("BATCH_LENGTH", 1);
  const int device = envi("NLP_DEVICE", 0);
  printf("OMP_NUM_THREADS=%d\n", threads);
  printf("Loading graph %s ...\n", file);
  // N1 / N2 on the device (default): the file's pairs parsed on all host
  // threads (nlp::readMtxPairs, as readMtxDoOmp), then ingest and every
  // deletion batch on the GPU (nlp_dcsr_*); NLP_HOST_INGEST=1 keeps the host
  // restatement (nlp/ingest.hxx) end to end.
  const bool host = envi("NLP_HOST_INGEST", 0) != 0;
  nlp::HostCsr x;
  nlp_dcsr* dx = nullptr;
  size_t xsize = 0;
  try {
    if (host) {
      x = nlp::readMtx(file);
      printGraph(x, "");
      if (!symmetric) {
        x = nlp::symmetrize(x);
        printGraph(x, " (symmetrize)");
      }
      x = nlp::removeSelfLoops(x);
      printGraph(x, " (removeSelfLoops)");
      xsize = x.size();
    } else {
      nlp::MtxPairs mp = nlp::readMtxPairs(file);
      nlp::check(nlp_dcsr_ingest(mp.src.empty() ? nullptr : mp.src.data(), mp.dst.empty() ? nullptr : mp.dst.data(),
                                 mp.src.size(), mp.n, symmetric ? 1 : 0, device, &dx),
                 "nlp_dcsr_ingest");
      uint64_t span = 0, nnz = 0, rs = 0, ss = 0;
      nlp::check(nlp_dcsr_info(dx, &span, &nnz, &rs, &ss), "nlp_dcsr_info");
      printf("order: %llu size: %llu [directed] {}\n", (unsigned long long)(span - 1), (unsigned long long)rs);
      if (!symmetric)
        printf("order: %llu size: %llu [directed] {} (symmetrize)\n", (unsigned long long)(span - 1),
               (unsigned long long)ss);
      printf("order: %llu size: %llu [directed] {} (removeSelfLoops)\n", (unsigned long long)(span - 1),
             (unsigned long long)nnz);
      xsize = nnz;
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "nlp_main: %s\n", e.what());
    return 1;
  }
  std::default_random_engine rnd;
  uint32_t seed = getenv("NLP_SEED") ? (uint32_t)strtoul(getenv("NLP_SEED"), nullptr, 10) : std::random_device()();
  rnd.seed(seed);
  uint32_t rng = seed;  // the device deletions continue one minstd_rand0 engine through its state
  std::vector<const Metric*> metrics;
  for (const auto& m : envlist("NLP_METRICS", "CN,JAC,SOR,SAL,HPI,HDI,LHN,AA,RA"))
    for (const auto& mm : METRICS)
      if (m == mm.name) metrics.push_back(&mm);
  std::vector<uint32_t> hubs;
  for (const auto& h : envlist("NLP_HUBS", "0,2,4,8,16,32,64,128,256,512,1024")) hubs.push_back((uint32_t)atoi(h.c_str()));
  const double dEnd = envd("BATCH_DELETIONS_END", 0.1);
  const char* dStep = getenv("BATCH_DELETIONS_STEP");
  for (double d = envd("BATCH_DELETIONS_BEGIN", 0.0001);;) {  // runBatches, main.cxx:157-179
    for (int r = 0; r < repeatBatch; ++r) {
      nlp::HostCsr y;
      if (host) y = x;
      const nlp_dcsr* cur = dx;  // device route: the batch graph (dx itself before the first batch)
      for (int seq = 0; seq < batchLength; ++seq) {
        const size_t batch = (size_t)(d * xsize / 2);
        std::vector<uint32_t> du, dv;
        nlp_graph* gh = nullptr;
        if (host) {
          auto del = nlp::generateEdgeDeletions(rnd, y, batch, 1, y.span() - 1, true);
          nlp::tidyDeletions(del, y);
          y = nlp::applyDeletions(y, del);
          du.resize(del.size());
          dv.resize(del.size());
          for (size_t i = 0; i < del.size(); ++i) { du[i] = del[i].first; dv[i] = del[i].second; }
        } else {
          nlp_dcsr* nx = nullptr;
          du.resize(2 * batch);
          dv.resize(2 * batch);
          uint64_t nd = 0;
          nlp::check(nlp_dcsr_delete_batch(cur, batch, &rng, &nx, du.data(), dv.data(), du.size(), &nd),
                     "nlp_dcsr_delete_batch");
          du.resize(nd);
          dv.resize(nd);
          if (cur != dx) nlp_dcsr_destroy(const_cast<nlp_dcsr*>(cur));
          cur = nx;
        }
        if (du.empty()) continue;  // main.cxx:209
        const auto tc0 = std::chrono::steady_clock::now();
        if (host) nlp::check(nlp_graph_create(y.off.data(), y.keys.empty() ? nullptr : y.keys.data(), y.span(), device, &gh),
                             "nlp_graph_create");
        else nlp::check(nlp_graph_create_dcsr(cur, &gh), "nlp_graph_create_dcsr");
        nlp::HipGraph hg(gh);
        {  // the per-graph build the 99 calls share (not a main.cxx line: process.js skips it)
          const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count();
          const char* names[32];
          double pms[32], alloc = 0;
          uint32_t np = 0;
          nlp::check(nlp_graph_build_phases(gh, 32, &np, names, pms, &alloc), "nlp_graph_build_phases");
          printf("graph build: %.1f ms (hipMalloc %.1f ms;", ms, alloc);
          for (uint32_t i = 0; i < np && i < 32; ++i) printf(" %s %.1f", names[i], pms[i]);
          printf(")\n");
          fflush(stdout);
        }
        nlp::check(nlp_set_truth(hg.get(), du.data(), dv.data(), du.size()), "nlp_set_truth");
        struct Del { size_t n; size_t size() const { return n; } } del{du.size()};
        const size_t k = del.size() / 2;  // insertions0.size() / 2 (main.cxx:50)
        for (const Metric* m : metrics) {
          for (uint32_t H : hubs) {
            auto p1 = nlp::predictLinksHip<uint32_t, float>(hg, m->id, H, PredictLinkOptions<float>(repeat, k));
            uint64_t common = 0;
            nlp::check(nlp_last_common(hg.get(), &common), "nlp_last_common");
            const double precision = double(common) / std::max<size_t>(2 * p1.edges.size(), 1);  // main.cxx:200
            const double recall = double(common) / std::max<size_t>(del.size(), 1);               // main.cxx:201
            printf("{-%.3e/+%.3e batchf, %03d threads} -> {%09.1fms, %09.1fms scoring, %.3e precision, %.3e recall} "
                   "%s%u\n",
                   0.0, d, threads, p1.time, p1.scoringTime, precision, recall, m->func, H);
            fflush(stdout);
          }
        }
      }
      if (cur != dx) nlp_dcsr_destroy(const_cast<nlp_dcsr*>(cur));
    }
    if (d >= dEnd) break;
    d = std::min(step(d, dStep), dEnd);
  }
  if (dx) nlp_dcsr_destroy(dx);
  printf("\n");
  return 0;
}
