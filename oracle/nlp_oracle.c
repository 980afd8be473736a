/*
 * nlp_oracle.c -- CPU restatement of the reference's link-prediction hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the *checker*: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path (libnlp.so, HIP) never links or calls it.
 *
 * Parity status: PINNED.  tests/golden/ holds fixtures produced by the real
 * reference (oracle/ref_driver.cxx compiled against /root/reference/inc by
 * oracle/Makefile, see tests/golden/make_golden.py); tests/test_oracle_golden.py
 * checks this restatement against them (candidate multisets bit-exact, top-k
 * above-boundary sets bit-exact, ties inside the reference's tie set).
 *
 * What it restates (all citations are /root/reference paths):
 *   - predictLinksWithIntersectionLoopU        inc/predict.hxx:214-265
 *       dense per-u counter table + touched list, hub filter deg(v) > H skip
 *       (predict.hxx:227), second-hop filter w > u (predict.hxx:221),
 *       first-order exclusion (predict.hxx:232-233), score <= minScore skip
 *       (predict.hxx:237)
 *   - predictScanEdgesBasicU / predictScanEdgesU inc/predict.hxx:153-179
 *   - predictClearScanW                         inc/predict.hxx:187-192
 *   - the nine metric score/update lambdas      inc/predict.hxx:502-831
 *   - the MAXFACTOR2 clause of ft (predict.hxx:221,295): with F > 0 a
 *     second-hop w is counted only when deg(w) <= F * deg(u) (its
 *     deg(u) <= F * deg(u) clause always holds for F >= 1)
 *   - degree() counts duplicate adjacency entries (Graph.hxx:167-169,
 *     _bitset.hxx:53), so every list is treated as a sorted multiset.
 *
 * Where the reference is nondeterministic (ties at the k-th score, SURVEY
 * Appendix A.1) or undefined (OpenMP dummy-heap read when candidates < k,
 * A.2; NaN scores, A.4), this restatement uses the canonical contract that the
 * GPU path also implements:
 *     order = (score key descending, u ascending, w ascending)
 *     NaN scores are kept (they pass `score <= minScore`, predict.hxx:237) and
 *     rank below every non-NaN score; -0.0 ranks equal to +0.0.
 *     fewer than maxEdges candidates -> return all of them (sequential
 *     reference behaviour, predict.hxx:358-374).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

enum {
  NLPO_CN = 0,   /* predictLinksCommonNeighbors          predict.hxx:502 */
  NLPO_JAC = 1,  /* predictLinksJaccardCoefficient       predict.hxx:540 */
  NLPO_SOR = 2,  /* predictLinksSorensenIndex            predict.hxx:578 */
  NLPO_SAL = 3,  /* predictLinksSaltonCosineSimilarity   predict.hxx:616 */
  NLPO_HPI = 4,  /* predictLinksHubPromoted              predict.hxx:654 */
  NLPO_HDI = 5,  /* predictLinksHubDepressed             predict.hxx:692 */
  NLPO_LHN = 6,  /* predictLinksLeichtHolmeNermanScore   predict.hxx:730 */
  NLPO_AA = 7,   /* predictLinksAdamicAdarCoefficient    predict.hxx:768 */
  NLPO_RA = 8    /* predictLinksResourceAllocationScore  predict.hxx:808 */
};

/* Order-preserving map float -> uint32 (larger score -> larger key).
 * NaN -> 0 (ranks last); -0.0 -> key of +0.0. */
uint32_t nlpo_score_key(float s) {
  uint32_t b;
  if (s != s) return 0u;
  if (s == 0.0f) s = 0.0f;
  memcpy(&b, &s, 4);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

/* Score of a basic (count) metric, predict.hxx:504-749.  du, dw are size_t
 * degrees (Graph.hxx:167), c is the uint32 wedge count (VT = K). */
static float score_basic(int metric, uint32_t c, uint64_t du, uint64_t dw) {
  float fc = (float)c;
  switch (metric) {
    case NLPO_CN:  return fc;                                   /* W(Nuv) */
    case NLPO_JAC: return fc / (float)(du + dw - (uint64_t)c);  /* size_t wrap kept */
    case NLPO_SOR: return fc / (float)(du + dw);
    case NLPO_SAL: return (float)((double)fc / sqrt((double)(du * dw)));
    case NLPO_HPI: return fc / (float)(du < dw ? du : dw);
    case NLPO_HDI: return fc / (float)(du < dw ? dw : du);
    case NLPO_LHN: return fc / (float)(du * dw);
    default: return 0.0f;
  }
}

/* Per-intermediate contribution of AA / RA (predict.hxx:770, 810), where the
 * lambda's `u` argument is the intermediate vertex v. */
static double contrib(int metric, uint64_t dv) {
  return metric == NLPO_AA ? 1.0 / log((double)dv) : 1.0 / (double)dv;
}

typedef struct {
  uint32_t u, w;
  float score;
  uint32_t key;
} cand_t;

typedef struct {
  cand_t *a;
  size_t n, cap;
} cvec_t;

static int cvec_push(cvec_t *v, cand_t c) {
  if (v->n == v->cap) {
    size_t nc = v->cap ? v->cap * 2 : 1024;
    cand_t *na = (cand_t *)realloc(v->a, nc * sizeof(cand_t));
    if (!na) return -1;
    v->a = na; v->cap = nc;
  }
  v->a[v->n++] = c;
  return 0;
}

static int cmp_u32(const void *x, const void *y) {
  uint32_t a = *(const uint32_t *)x, b = *(const uint32_t *)y;
  return (a > b) - (a < b);
}

/* Canonical order: key desc, u asc, w asc. */
static int cmp_cand(const void *x, const void *y) {
  const cand_t *a = (const cand_t *)x, *b = (const cand_t *)y;
  if (a->key != b->key) return a->key < b->key ? 1 : -1;
  if (a->u != b->u) return a->u < b->u ? -1 : 1;
  if (a->w != b->w) return a->w < b->w ? -1 : 1;
  return 0;
}

/* Per-source scratch of the reference's loop (predict.hxx:280-283): the dense
 * counter table veout (count or float accumulator) and the touched list vedgs. */
typedef struct {
  uint32_t *cnt;
  float *acc;
  uint32_t *touched;
} tables_t;

static int tables_alloc(tables_t *t, uint64_t span, int custom) {
  t->cnt = (uint32_t *)calloc(span ? span : 1, sizeof(uint32_t));
  t->acc = custom ? (float *)calloc(span ? span : 1, sizeof(float)) : NULL;
  t->touched = (uint32_t *)malloc((span ? span : 1) * sizeof(uint32_t));
  return (!t->cnt || !t->touched || (custom && !t->acc)) ? -1 : 0;
}

static void tables_free(tables_t *t) {
  free(t->cnt); free(t->acc); free(t->touched);
  t->cnt = NULL; t->acc = NULL; t->touched = NULL;
}

typedef int (*emit_fn)(void *arg, uint32_t u, uint32_t w, float s, uint32_t key);

/*
 * One source u of predictLinksWithIntersectionLoopU (predict.hxx:214-265):
 * emits every candidate (u, w, score) with score > min_score (or NaN) in
 * ascending w.  Adds the wedges the reference scans (SURVEY §8(d) W_H) and
 * those with w > u (the wedges that reach the counter table).
 */
static int scan_source(const uint64_t *off, const uint32_t *keys, uint64_t span,
                       int metric, uint32_t hub, uint32_t maxf2, float min_score, uint64_t u,
                       tables_t *tb, emit_fn emit, void *arg, uint64_t *wedges, uint64_t *wedges_gt) {
  int custom = (metric == NLPO_AA || metric == NLPO_RA);
  uint32_t *cnt = tb->cnt, *touched = tb->touched;
  float *acc = tb->acc;
  size_t nt = 0;
  uint64_t du = off[u + 1] - off[u];
  /* wedge scan: predict.hxx:224-230 -> 153-179 */
  for (uint64_t i = off[u]; i < off[u + 1]; ++i) {
    uint32_t v = keys[i];
    uint64_t dv = v < span ? off[v + 1] - off[v] : 0;
    if (hub && dv > hub) continue;                /* predict.hxx:227 */
    double c = custom ? contrib(metric, dv) : 0.0;
    for (uint64_t j = off[v]; j < off[v + 1]; ++j) {
      uint32_t w = keys[j];
      ++*wedges;
      if (!(w > u)) continue;                      /* ft: predict.hxx:221 */
      ++*wedges_gt;
      if (maxf2 && (w < span ? off[w + 1] - off[w] : 0) > (uint64_t)maxf2 * du)
        continue;                                  /* ft, MAXFACTOR2 clause */
      if (custom) {
        if (!acc[w]) touched[nt++] = w;            /* predict.hxx:176 */
        acc[w] = (float)((double)acc[w] + c);      /* fu: entry += 1.0/..  */
      } else {
        if (!cnt[w]) touched[nt++] = w;            /* predict.hxx:157 */
        ++cnt[w];
      }
    }
  }
  /* first-order exclusion, predict.hxx:232-233 */
  if (custom) acc[u] = 0.0f; else cnt[u] = 0;
  for (uint64_t i = off[u]; i < off[u + 1]; ++i) {
    if (custom) acc[keys[i]] = 0.0f; else cnt[keys[i]] = 0;
  }
  /* canonical w order inside u (the reference scores in first-touch order,
     which only matters for ties, A.1) */
  qsort(touched, nt, sizeof(uint32_t), cmp_u32);
  int rc = 0;
  for (size_t t = 0; t < nt; ++t) {
    uint32_t w = touched[t];
    float s;
    if (custom) s = acc[w];                        /* fs = W(Nuv) */
    else {
      uint64_t dw = w < span ? off[w + 1] - off[w] : 0;
      s = score_basic(metric, cnt[w], du, dw);
    }
    if (custom) acc[w] = 0.0f; else cnt[w] = 0;    /* predictClearScanW 187-192 */
    if (s <= min_score) continue;                  /* predict.hxx:237 (NaN passes) */
    if (!rc && emit(arg, (uint32_t)u, w, s, nlpo_score_key(s))) rc = -1;
  }
  return rc;
}

static int emit_push(void *arg, uint32_t u, uint32_t w, float s, uint32_t key) {
  cand_t cd = {u, w, s, key};
  return cvec_push((cvec_t *)arg, cd);
}

/*
 * Enumerate every candidate (u, w, score) with score > min_score (or NaN) for
 * u in [u_begin, u_end), in (u asc, w asc) order.  Returns 0 on success.
 */
static int enumerate(const uint64_t *off, const uint32_t *keys, uint64_t span,
                     int metric, uint32_t hub, uint32_t maxf2, float min_score,
                     uint64_t u_begin, uint64_t u_end, cvec_t *out,
                     uint64_t *wedges_out, uint64_t *wedges_gt_out) {
  int custom = (metric == NLPO_AA || metric == NLPO_RA);
  tables_t tb;
  uint64_t wedges = 0, wedges_gt = 0;
  if (tables_alloc(&tb, span, custom)) { tables_free(&tb); return -1; }
  for (uint64_t u = u_begin; u < u_end && u < span; ++u) {
    if (scan_source(off, keys, span, metric, hub, maxf2, min_score, u, &tb, emit_push, out, &wedges, &wedges_gt)) {
      tables_free(&tb);
      return -1;
    }
  }
  tables_free(&tb);
  if (wedges_out) *wedges_out = wedges;
  if (wedges_gt_out) *wedges_gt_out = wedges_gt;
  return 0;
}

/*
 * Canonical top-k.  Writes at most max_edges tuples (score desc, u asc, w asc)
 * into out_u/out_w/out_score (caller-owned, may be NULL when max_edges == 0)
 * and the number written into *out_count.  *n_candidates gets the number of
 * candidates that passed the score filter, *n_nan those with NaN score,
 * *n_wedges the wedges scanned.  Returns 0 on success, -1 on allocation failure.
 */
int nlpo_predict_range2(const uint64_t *off, const uint32_t *keys, uint64_t span,
                        int metric, uint32_t hub, uint32_t maxf2, float min_score, uint64_t max_edges,
                        uint64_t u_begin, uint64_t u_end,
                        uint32_t *out_u, uint32_t *out_w, float *out_score,
                        uint64_t *out_count, uint64_t *n_candidates, uint64_t *n_nan,
                        uint64_t *n_wedges, uint64_t *n_wedges_gt) {
  cvec_t c = {0, 0, 0};
  if (enumerate(off, keys, span, metric, hub, maxf2, min_score, u_begin, u_end, &c, n_wedges, n_wedges_gt)) {
    free(c.a); return -1;
  }
  uint64_t nn = 0;
  for (size_t i = 0; i < c.n; ++i) nn += (c.a[i].key == 0);
  if (n_candidates) *n_candidates = c.n;
  if (n_nan) *n_nan = nn;
  uint64_t take = c.n < max_edges ? c.n : max_edges;
  if (take == 0) c.n = 0;
  if (take < c.n) {
    /* threshold = take-th largest key; candidates are in (u,w) order, so the
       first `quota` ties in that order are the canonical tie fill. */
    uint32_t *hi = (uint32_t *)calloc(65536, sizeof(uint32_t));
    uint32_t *lo = (uint32_t *)calloc(65536, sizeof(uint32_t));
    if (!hi || !lo) { free(hi); free(lo); free(c.a); return -1; }
    for (size_t i = 0; i < c.n; ++i) hi[c.a[i].key >> 16]++;
    uint64_t acc = 0; int b = 65535;
    for (; b >= 0; --b) { if (acc + hi[b] >= take) break; acc += hi[b]; }
    for (size_t i = 0; i < c.n; ++i) if ((c.a[i].key >> 16) == (uint32_t)b) lo[c.a[i].key & 0xffff]++;
    int l = 65535;
    for (; l >= 0; --l) { if (acc + lo[l] >= take) break; acc += lo[l]; }
    uint32_t kth = ((uint32_t)b << 16) | (uint32_t)l;
    uint64_t quota = take - acc;  /* ties to keep */
    size_t j = 0;
    for (size_t i = 0; i < c.n; ++i) {
      if (c.a[i].key > kth) c.a[j++] = c.a[i];
      else if (c.a[i].key == kth && quota) { c.a[j++] = c.a[i]; --quota; }
    }
    c.n = j;
    free(hi); free(lo);
  }
  qsort(c.a, c.n, sizeof(cand_t), cmp_cand);
  if (c.n > take) c.n = take;
  for (size_t i = 0; i < c.n; ++i) {
    if (out_u) out_u[i] = c.a[i].u;
    if (out_w) out_w[i] = c.a[i].w;
    if (out_score) out_score[i] = c.a[i].score;
  }
  if (out_count) *out_count = c.n;
  free(c.a);
  return 0;
}

int nlpo_predict_range(const uint64_t *off, const uint32_t *keys, uint64_t span,
                       int metric, uint32_t hub, float min_score, uint64_t max_edges,
                       uint64_t u_begin, uint64_t u_end,
                       uint32_t *out_u, uint32_t *out_w, float *out_score,
                       uint64_t *out_count, uint64_t *n_candidates, uint64_t *n_nan,
                       uint64_t *n_wedges, uint64_t *n_wedges_gt) {
  return nlpo_predict_range2(off, keys, span, metric, hub, 0, min_score, max_edges, u_begin, u_end,
                             out_u, out_w, out_score, out_count, n_candidates, n_nan, n_wedges, n_wedges_gt);
}

int nlpo_predict(const uint64_t *off, const uint32_t *keys, uint64_t span,
                 int metric, uint32_t hub, float min_score, uint64_t max_edges,
                 uint32_t *out_u, uint32_t *out_w, float *out_score,
                 uint64_t *out_count, uint64_t *n_candidates, uint64_t *n_nan,
                 uint64_t *n_wedges) {
  return nlpo_predict_range(off, keys, span, metric, hub, min_score, max_edges, 0, span,
                            out_u, out_w, out_score, out_count, n_candidates, n_nan, n_wedges, NULL);
}

/* Number of candidates (score > min_score or NaN) -- sizing helper for tests. */
int nlpo_count_candidates(const uint64_t *off, const uint32_t *keys, uint64_t span,
                          int metric, uint32_t hub, float min_score,
                          uint64_t *n_candidates, uint64_t *n_wedges) {
  return nlpo_predict(off, keys, span, metric, hub, min_score, 0, NULL, NULL, NULL,
                      NULL, n_candidates, NULL, n_wedges);
}

/* ------------------------------------------------------------------------
 * Parallel restatement for the full-size configs.
 *
 * The same per-source scan (scan_source, predict.hxx:214-265) over the source
 * range cut into chunks of consecutive u, run by OpenMP threads with one set
 * of tables each -- the reference's own parallelisation (predict.hxx:284-339,
 * one table per thread), without its per-thread heaps.  Candidates are never
 * all stored; four passes over the sources:
 *   A  count the candidates, histogram of key >> 16     -> take = min(k, C)
 *   B  histogram of key & 0xffff inside the boundary bin -> k-th key, tie quota
 *   C  per chunk: candidates above the k-th key, ties at it
 *   D  per chunk: write the kept ones (all above, ties while the chunk's share
 *      of the quota lasts -- chunks ascend in u, so this is the canonical
 *      (u asc, w asc) tie fill) at the chunk's prefix offset
 * then a stable LSD radix sort by descending key puts the kept set in the
 * canonical order (score desc, u asc, w asc).  The digest (sum and xor of
 * nlpo_edge_hash over the kept set) is order-free, for checks that do not
 * copy the result.
 * ------------------------------------------------------------------------ */
#ifdef _OPENMP
#include <omp.h>
#endif

/* splitmix64 finaliser */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Hash of one predicted link: (u, w) and the score bits (NaN canonicalised). */
uint64_t nlpo_edge_hash(uint32_t u, uint32_t w, float s) {
  uint32_t b;
  if (s != s) b = 0x7fc00000u;
  else memcpy(&b, &s, 4);
  return mix64((((uint64_t)u << 32) | w) ^ ((uint64_t)b * 0x9E3779B97F4A7C15ull));
}

typedef struct {
  uint64_t *hist;       /* pass A: 65536 bins of key >> 16; pass B: of key & 0xffff */
  uint32_t hi;          /* pass B: the boundary bin */
  uint32_t kth;         /* passes C, D */
  uint64_t above, ties; /* pass C: this chunk's counts */
  uint64_t ncand, nnan;
  cand_t *dst;          /* pass D: the chunk's slice */
  uint64_t quota;       /* pass D: ties this chunk keeps */
  uint64_t n;           /* pass D: written */
  uint64_t dsum, dxor;
  int all;              /* pass D: keep every candidate */
} pass_t;

static int emit_a(void *arg, uint32_t u, uint32_t w, float s, uint32_t key) {
  pass_t *p = (pass_t *)arg;
  (void)u; (void)w; (void)s;
  p->hist[key >> 16]++;
  p->ncand++;
  p->nnan += (key == 0);
  return 0;
}

static int emit_b(void *arg, uint32_t u, uint32_t w, float s, uint32_t key) {
  pass_t *p = (pass_t *)arg;
  (void)u; (void)w; (void)s;
  if ((key >> 16) == p->hi) p->hist[key & 0xffff]++;
  return 0;
}

static int emit_c(void *arg, uint32_t u, uint32_t w, float s, uint32_t key) {
  pass_t *p = (pass_t *)arg;
  (void)u; (void)w; (void)s;
  if (key > p->kth) p->above++;
  else if (key == p->kth) p->ties++;
  return 0;
}

static int emit_d(void *arg, uint32_t u, uint32_t w, float s, uint32_t key) {
  pass_t *p = (pass_t *)arg;
  if (p->all || key > p->kth || (key == p->kth && p->quota)) {
    if (!p->all && key == p->kth) p->quota--;
    cand_t c = {u, w, s, key};
    p->dst[p->n++] = c;
    uint64_t h = nlpo_edge_hash(u, w, s);
    p->dsum += h;
    p->dxor ^= h;
  }
  return 0;
}

/* Stable LSD radix sort by descending key (the input is in (u, w) order). */
static int sort_desc(cand_t *a, uint64_t n) {
  if (n < 2) return 0;
  cand_t *tmp = (cand_t *)malloc(n * sizeof(cand_t));
  if (!tmp) return -1;
  cand_t *src = a, *dst = tmp;
  for (int sh = 0; sh < 32; sh += 8) {
    uint64_t cnt[257];
    memset(cnt, 0, sizeof cnt);
    for (uint64_t i = 0; i < n; ++i) cnt[((~src[i].key) >> sh & 255) + 1]++;
    for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
    for (uint64_t i = 0; i < n; ++i) dst[cnt[(~src[i].key) >> sh & 255]++] = src[i];
    cand_t *t = src; src = dst; dst = t;
  }
  /* four passes: the result is back in a */
  free(tmp);
  return 0;
}

/*
 * nlpo_predict_par: canonical top max_edges of [u_begin, u_end) with `threads`
 * OpenMP threads (0 = the OpenMP default).  out_u/out_w/out_score (nullable)
 * receive the result in canonical order.  stats[0..7] = out_count,
 * candidates, NaN candidates, wedges, wedges (w > u), k-th key, digest sum,
 * digest xor.  Returns 0, or -1 on allocation failure.
 */
int nlpo_predict_par(const uint64_t *off, const uint32_t *keys, uint64_t span,
                     int metric, uint32_t hub, uint32_t maxf2, float min_score, uint64_t max_edges,
                     uint64_t u_begin, uint64_t u_end, int threads,
                     uint32_t *out_u, uint32_t *out_w, float *out_score, uint64_t *stats) {
  int custom = (metric == NLPO_AA || metric == NLPO_RA);
  if (u_end > span) u_end = span;
  if (u_begin > u_end) u_begin = u_end;
  for (int i = 0; i < 8; ++i) stats[i] = 0;
  int T = 1;
#ifdef _OPENMP
  T = threads > 0 ? threads : omp_get_max_threads();
#else
  (void)threads;
#endif
  const uint64_t nu = u_end - u_begin;
  const uint64_t nch = nu == 0 ? 1 : (nu < 16384 ? nu : 16384);
  uint64_t *above = (uint64_t *)calloc(nch, 8), *ties = (uint64_t *)calloc(nch, 8);
  uint64_t *hist = (uint64_t *)calloc((size_t)T * 65536, 8);
  tables_t *tb = (tables_t *)calloc(T, sizeof(tables_t));
  int fail = !above || !ties || !hist || !tb;
  for (int t = 0; t < T && !fail; ++t) fail = tables_alloc(&tb[t], span, custom);
  uint64_t wedges = 0, wedges_gt = 0, ncand = 0, nnan = 0;
  cand_t *kept = NULL;
#define CHUNK_LO(c) (u_begin + nu * (uint64_t)(c) / nch)
#define CHUNK_HI(c) (u_begin + nu * (uint64_t)((c) + 1) / nch)
  /* pass A */
  if (!fail) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(T) reduction(+ : wedges, wedges_gt, ncand, nnan)
    for (int64_t c = 0; c < (int64_t)nch; ++c) {
      int t = 0;
#ifdef _OPENMP
      t = omp_get_thread_num();
#endif
      pass_t p;
      memset(&p, 0, sizeof p);
      p.hist = hist + (size_t)t * 65536;
      for (uint64_t u = CHUNK_LO(c); u < CHUNK_HI(c); ++u)
        scan_source(off, keys, span, metric, hub, maxf2, min_score, u, &tb[t], emit_a, &p, &wedges, &wedges_gt);
      above[c] = p.ncand;  /* all kept when take == ncand: pass C is skipped */
      ncand += p.ncand;
      nnan += p.nnan;
    }
  }
  uint64_t take = ncand < max_edges ? ncand : max_edges;
  uint32_t kth = 0;
  uint64_t quota = 0;
  if (!fail && take > 0 && take < ncand) {
    uint64_t acc = 0;
    int b = 65535;
    for (; b >= 0; --b) {
      uint64_t h = 0;
      for (int t = 0; t < T; ++t) h += hist[(size_t)t * 65536 + b];
      if (acc + h >= take) break;
      acc += h;
    }
    memset(hist, 0, (size_t)T * 65536 * 8);
    uint64_t dummy0 = 0, dummy1 = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(T) reduction(+ : dummy0, dummy1)
    for (int64_t c = 0; c < (int64_t)nch; ++c) {
      int t = 0;
#ifdef _OPENMP
      t = omp_get_thread_num();
#endif
      pass_t p;
      memset(&p, 0, sizeof p);
      p.hist = hist + (size_t)t * 65536;
      p.hi = (uint32_t)b;
      for (uint64_t u = CHUNK_LO(c); u < CHUNK_HI(c); ++u)
        scan_source(off, keys, span, metric, hub, maxf2, min_score, u, &tb[t], emit_b, &p, &dummy0, &dummy1);
    }
    int l = 65535;
    for (; l >= 0; --l) {
      uint64_t h = 0;
      for (int t = 0; t < T; ++t) h += hist[(size_t)t * 65536 + l];
      if (acc + h >= take) break;
      acc += h;
    }
    kth = ((uint32_t)b << 16) | (uint32_t)l;
    quota = take - acc;
  }
  /* passes C and D (with take == ncand every candidate is kept: kth = 0 and
     all ties -- key 0 = NaN -- fit the quota) */
  if (!fail && take > 0) {
    if (take == ncand) quota = 0;  /* above[c] (pass A) already counts every candidate, NaN included */
    uint64_t dummy0 = 0, dummy1 = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(T) reduction(+ : dummy0, dummy1)
    for (int64_t c = 0; c < (int64_t)(take < ncand ? nch : 0); ++c) {
      int t = 0;
#ifdef _OPENMP
      t = omp_get_thread_num();
#endif
      pass_t p;
      memset(&p, 0, sizeof p);
      p.kth = kth;
      for (uint64_t u = CHUNK_LO(c); u < CHUNK_HI(c); ++u)
        scan_source(off, keys, span, metric, hub, maxf2, min_score, u, &tb[t], emit_c, &p, &dummy0, &dummy1);
      above[c] = p.above;
      ties[c] = p.ties;
    }
    kept = (cand_t *)malloc((take ? take : 1) * sizeof(cand_t));
    fail = !kept;
  }
  uint64_t dsum = 0, dxor = 0;
  if (!fail && take > 0) {
    /* each chunk's slice and tie share, in chunk (= u) order */
    uint64_t *base = (uint64_t *)malloc(nch * 8), *share = (uint64_t *)malloc(nch * 8);
    fail = !base || !share;
    if (!fail) {
      uint64_t pos = 0, q = quota;
      for (uint64_t c = 0; c < nch; ++c) {
        share[c] = ties[c] < q ? ties[c] : q;
        q -= share[c];
        base[c] = pos;
        pos += above[c] + share[c];
      }
      uint64_t dummy0 = 0, dummy1 = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(T) reduction(+ : dummy0, dummy1, dsum) reduction(^ : dxor)
      for (int64_t c = 0; c < (int64_t)nch; ++c) {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        pass_t p;
        memset(&p, 0, sizeof p);
        p.kth = kth;
        p.quota = share[c];
        p.all = take == ncand;
        p.dst = kept + base[c];
        for (uint64_t u = CHUNK_LO(c); u < CHUNK_HI(c); ++u)
          scan_source(off, keys, span, metric, hub, maxf2, min_score, u, &tb[t], emit_d, &p, &dummy0, &dummy1);
        dsum += p.dsum;
        dxor ^= p.dxor;
      }
      if (out_u || out_w || out_score) fail = sort_desc(kept, take);
      for (uint64_t i = 0; i < take && !fail; ++i) {
        if (out_u) out_u[i] = kept[i].u;
        if (out_w) out_w[i] = kept[i].w;
        if (out_score) out_score[i] = kept[i].score;
      }
    }
    free(base);
    free(share);
  }
#undef CHUNK_LO
#undef CHUNK_HI
  for (int t = 0; tb && t < T; ++t) tables_free(&tb[t]);
  free(tb); free(hist); free(above); free(ties); free(kept);
  if (fail) return -1;
  stats[0] = take;
  stats[1] = ncand;
  stats[2] = nnan;
  stats[3] = wedges;
  stats[4] = wedges_gt;
  stats[5] = kth;
  stats[6] = dsum;
  stats[7] = dxor;
  return 0;
}

/* Wedges (u, v, w) with w > u of the sources [ua, ub): the count of the
 * reference's wedge loop (predict.hxx:284-304 -> 153-160: every v of N(u)
 * with deg v <= H, or all for H = 0, every w of N(v) with w > u), found per
 * (u, v) entry by one binary search of the sorted list N(v) instead of a walk
 * -- O(entries log deg) for ranges whose walk would take minutes (the C5
 * shards' property test).  OpenMP over sources when built with it. */
uint64_t nlpo_wedges_gt(const uint64_t *off, const uint32_t *keys, uint64_t span, uint32_t hub, uint64_t ua,
                        uint64_t ub, int threads) {
  uint64_t total = 0;
  if (ub > span) ub = span;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : total)
#endif
  for (long long uu = (long long)ua; uu < (long long)ub; ++uu) {
    const uint64_t u = (uint64_t)uu;
    for (uint64_t i = off[u]; i < off[u + 1]; ++i) {
      const uint32_t v = keys[i];
      if (v >= span) continue;
      const uint64_t lo0 = off[v], hi0 = off[v + 1];
      if (hub && hi0 - lo0 > hub) continue;        /* predict.hxx:298-301 */
      uint64_t lo = lo0, hi = hi0;                 /* first entry of N(v) above u */
      while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if (keys[m] <= u) lo = m + 1; else hi = m;
      }
      total += hi0 - lo;
    }
  }
  return total;
}
