/*
 * nlp.h -- C-ABI of the MI355X (gfx950) neighborhood link-prediction engine
 * (libnlp.so).  Plain pointers and sizes only; no HIP or torch types.
 *
 * This is the drop-in boundary for the reference's hot path
 * (/root/reference/inc/predict.hxx).  The reference's entry points are C++
 * templates called from main.cxx:50:
 *
 *   template <int MINDEGREE1=4, int MAXFACTOR2=0, bool FORCEHEAP=false, class G, class W=float>
 *   auto predictLinks<Metric>Omp(const G& x, const PredictLinkOptions<W>& o={})
 *       -> PredictLinkResult<typename G::key_type, W>          (predict.hxx:519-831)
 *
 * Templates and lambdas cannot cross a C ABI, so the metric becomes an enum
 * (the nine built-in metrics, predict.hxx:502-831), MINDEGREE1 becomes the
 * runtime `hub_max_degree` (0 = IHub), PredictLinkOptions{repeat, maxEdges,
 * minScore} (predict.hxx:33-55) become arguments, and PredictLinkResult
 * {edges, time, scoringTime} (predict.hxx:65-102) becomes the caller-owned
 * `out` array plus nlp_timing.  The C++ header include/nlp/predict.hxx
 * rebuilds the reference's template API on top of these functions.
 *
 * Graph input = CSR of the reference's graph concept (Graph.hxx span /
 * forEachEdgeKey / degree, csr.hxx csrCreateOffsetsW / csrCreateEdgeKeysW):
 * offsets[span+1] (u64, like DiGraphCsr<..., O=size_t>), keys[nnz] (u32 vertex
 * ids, each adjacency list sorted ascending; duplicate entries are allowed and
 * counted, exactly like LazyBitset lists, _bitset.hxx:53,114).  Vertices with no
 * edges (including the reference's absent vertex 0) simply have empty rows.
 *
 * Output order is canonical: score descending, then u ascending, then v
 * ascending.  The reference's own tie order is thread-schedule dependent
 * (SURVEY.md Appendix A.1); its score multiset and above-boundary set are
 * reproduced bit-exactly.  Every output pair has u < v.
 *
 * Errors: the reference has none (everything noexcept, bad input is UB).  Every
 * function here returns an nlp_status and never throws or aborts.
 */
#ifndef NLP_H
#define NLP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  NLP_OK = 0,
  NLP_ERR_INVALID = 1,    /* bad argument or malformed CSR */
  NLP_ERR_DEVICE = 2,     /* HIP runtime / kernel failure */
  NLP_ERR_NOMEM = 3,      /* device or host allocation failed */
  NLP_ERR_NODEVICE = 4,   /* no usable gfx950 device */
  NLP_ERR_CAPACITY = 5,   /* caller buffer too small (see out_count) */
  NLP_ERR_RETRY = 6       /* nlp_sync: a call of the asynchronous batch needs a synchronous redo */
} nlp_status;

/* The nine similarity metrics of predict.hxx (enum order = main.cxx:212-220). */
typedef enum {
  NLP_CN = 0,   /* predictLinksCommonNeighbors[Omp]           predict.hxx:502,519 */
  NLP_JAC = 1,  /* predictLinksJaccardCoefficient[Omp]        predict.hxx:540,557 */
  NLP_SOR = 2,  /* predictLinksSorensenIndex[Omp]             predict.hxx:578,595 */
  NLP_SAL = 3,  /* predictLinksSaltonCosineSimilarity[Omp]    predict.hxx:616,633 */
  NLP_HPI = 4,  /* predictLinksHubPromoted[Omp]               predict.hxx:654,671 */
  NLP_HDI = 5,  /* predictLinksHubDepressed[Omp]              predict.hxx:692,709 */
  NLP_LHN = 6,  /* predictLinksLeichtHolmeNermanScore[Omp]    predict.hxx:730,747 */
  NLP_AA = 7,   /* predictLinksAdamicAdarCoefficient[Omp]     predict.hxx:768,786 */
  NLP_RA = 8    /* predictLinksResourceAllocationScore[Omp]   predict.hxx:808,826 */
} nlp_metric;

/* One predicted link: PredictLinkResult::edges element tuple<K,K,W>
 * (predict.hxx:69) with K = uint32_t, W = float. */
typedef struct {
  uint32_t u;
  uint32_t v;
  float score;
} nlp_edge;

/* Timing and counters of one predict call.  score_ms / total_ms correspond to
 * PredictLinkResult::scoringTime / time (predict.hxx:71-73, 466): score_ms is
 * averaged over `repeat` like measureDuration (_utility.hxx:345-352); select_ms
 * is the top-k selection + ordering (the reference's merge, predict.hxx:431-460);
 * copy_ms is the device->host copy of the result (not part of total_ms).  All
 * from HIP events on the device stream. */
typedef struct {
  float score_ms;
  float select_ms;
  float total_ms;
  float copy_ms;
  uint64_t wedges;          /* (u, v, w) wedges scanned, w > u  (SURVEY §8(d) W_H) */
  uint64_t candidates;      /* candidates with score > min_score (NaN included) */
  uint64_t nan_candidates;  /* of which NaN */
  uint32_t path;            /* 1 = intermediate-centric sort grouping, 2 = source-centric chunked sort,
                               3 = intermediate-centric radix grouping, 4 = source-centric hash
                               accumulation */
  uint32_t chunks;          /* source-range chunks used by paths 2 and 4 */
  float hot_ms;             /* device time of the dominant kernel (HIP events around its launch) */
  uint32_t graph_replay;    /* 1 when the call replayed a captured hipGraph */
  uint64_t hot_bytes;       /* algorithmic bytes of that launch */
  uint32_t hot_kernel;      /* which kernel hot_ms times: 1 k_sp_bucket, 2 k_sp_scan<F_Runs>,
                               3 k_group_tiles, 4 k_sp_survivors, 5 k_sp_expand, 6 k_sp_pass,
                               7 k_sp_runs, 8 k_sp_group, 9 k_sp_grouprun, 10 k_sp_exbucket,
                               11 k_hp_batch (path 4: all its launches of the call, times and bytes
                               summed), 12 k_sp_order_rank; 0 none.  Path 1's fused call reports
                               the longest of k_sp_exbucket, k_sp_grouprun, k_sp_order_rank */
  uint64_t call_bytes;      /* algorithmic bytes of ALL the call's kernels by the DESIGN.md §5 model
                               (paths 1 and 4; 0 when not modelled) -- what this call's own design
                               must move, beside SURVEY §8(d)'s bytes of the reference's scan */
  uint32_t order_route;     /* path 4: how the final order ran -- NLP_ORDER_FOLD8 (the last prune folded
                               into the 8-byte order), NLP_ORDER_FOLD_REFUSED (folded, the keys refused
                               the 8-byte order: pruned, then the 12-byte sort), NLP_ORDER_SORT8 / _SORT12
                               (pruned, then the 8-byte / 12-byte sort); 0 for the other paths; with
                               NLP_ORDER_RUNS added when the 8-byte order took its two-level form (LSD
                               passes over (rank, u), then every run of equal (rank, u) put in w order) */
} nlp_timing;
#define NLP_ORDER_FOLD8 1
#define NLP_ORDER_FOLD_REFUSED 2
#define NLP_ORDER_SORT8 3
#define NLP_ORDER_SORT12 4
#define NLP_ORDER_RUNS 16

typedef struct nlp_graph nlp_graph;

/* Upload a host CSR to `device` (HIP ordinal) and build the graph handle.
 * Inputs are borrowed for the duration of the call only.  The handle keeps the
 * CSR, degrees, the transposed adjacency (shared when the graph is symmetric)
 * and the Adamic-Adar / Resource-Allocation contribution tables resident in
 * HBM for its lifetime (main.cxx runs 99 predictions per graph). */
nlp_status nlp_graph_create(const uint64_t* offsets, const uint32_t* keys, uint64_t span,
                            int device, nlp_graph** out);

/* Same, from CSR arrays already resident on `device` (device pointers).  The
 * arrays are copied; `stream` (hipStream_t or NULL) orders the copy. */
nlp_status nlp_graph_create_device(const uint64_t* d_offsets, const uint32_t* d_keys, uint64_t span,
                                   uint64_t nnz, int device, void* stream, nlp_graph** out);

/* Multi-device graph: the reference's one OpenMP team over all source vertices
 * (predict.hxx:284-339, omp_get_max_threads() threads, predict.hxx:413) becomes
 * `ndev` partitions of the source range, partition p on HIP device devices[p]
 * (a device may appear several times: logical partitions sharing its
 * replica).  Every distinct device keeps a full replica of the graph (second-
 * hop lists are arbitrary).  The partitions are balanced by the wedge work of
 * the call's hub threshold (computed once per threshold).  A predict call runs
 * every partition's canonical top-k on its device (one host thread per
 * device), then selects the global top-k histogram-first (key histograms of
 * the partitions' lists give the k-th key and each partition's share, a prefix
 * of its list), copies only the shares to devices[0] (peer copies over xGMI)
 * and merges them there in one kernel -- the same result, bit for bit and in
 * the same order, as a single-device handle.  Device outputs (d_out of
 * nlp_predict_device*) live on devices[0].  nlp_predict_device_async is not
 * available on a multi-device handle (NLP_ERR_INVALID).  ndev <= NLP_MAX_PARTS. */
#define NLP_MAX_PARTS 64
nlp_status nlp_graph_create_multi(const uint64_t* offsets, const uint32_t* keys, uint64_t span,
                                  const int* devices, int ndev, nlp_graph** out);

/* Number of visible gfx950 devices (the C++ header's default device set). */
int nlp_device_count(void);

/* Partitions of a handle: *nparts (1 for a single-device handle) and, when
 * `bounds` is not NULL, the nparts + 1 source bounds used by the last
 * prediction (NLP_ERR_INVALID before the first prediction of a group). */
nlp_status nlp_graph_parts(const nlp_graph* g, int* nparts, uint64_t* bounds);

void nlp_graph_destroy(nlp_graph* g);

/* Graph properties: span (S), nnz (M), maximum degree, symmetric flag. */
nlp_status nlp_graph_info(const nlp_graph* g, uint64_t* span, uint64_t* nnz, uint32_t* max_degree,
                          int* symmetric);

/* Where the graph build went (no reference counterpart: the reference builds
 * nothing per graph beyond its DiGraph, and main.cxx times only the predict
 * calls, main.cxx:50 / predict.hxx:420-430).  *n receives the number of build
 * phases of the create call that made `g` (for a multi-device handle: its
 * first replica's); the first min(*n, cap) are written in build order as
 * (names[i], ms[i]): host wall time with the device stream drained at every
 * phase boundary, so the phases sum to the create call's time.  *alloc_ms
 * (may be NULL) is the part of that time spent inside hipMalloc.  Names:
 * upload, degrees, row_index, transpose, degree_class_index, entry_classes,
 * short_lists, membership_table, edge_filter, tables_and_setup. */
nlp_status nlp_graph_build_phases(const nlp_graph* g, uint32_t cap, uint32_t* n, const char** names, double* ms,
                                  double* alloc_ms);

/* Measurement hook (no reference counterpart): the sort path's stage whose
 * launch nlp_timing.hot_ms times with HIP events recorded around it on the
 * call's stream (stage 2 = k_sp_exbucket of the fused call); -1 (the default)
 * restores the kernels' own low-overhead stamps.  Results are unchanged. */
nlp_status nlp_set_hot_stage(nlp_graph* g, int stage);

/* predictLinks<Metric>Omp<hub_max_degree>(G, {repeat, max_edges, min_score}).
 * `out` is a caller-owned HOST array of at least min(max_edges, number of
 * candidates) entries, or NULL.  *out_count receives the number of predicted
 * links (< max_edges when there are fewer candidates; the reference's
 * OpenMP merge reads out of bounds in that case).
 * max_edges = UINT64_MAX means "all candidates".  Count query: pass
 * out = NULL (any max_edges, typically UINT64_MAX); the links are computed and
 * kept on the device, *out_count holds their number, and nlp_copy_last
 * fetches them without predicting again.  max_edges = 0 predicts nothing
 * (*out_count = 0, t->candidates = 0), like the reference's `o.maxEdges > 0`
 * guard (predict.hxx:367,429). */
nlp_status nlp_predict(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, float min_score,
                       uint64_t max_edges, int repeat, nlp_edge* out, uint64_t* out_count,
                       nlp_timing* t);

/* Same with the reference's MAXFACTOR2 template parameter (predict.hxx:221,295):
 * max_factor2 > 0 keeps a second-hop candidate w of source u only when
 * deg(w) <= max_factor2 * deg(u) (the clause deg(u) <= MAXFACTOR2 * deg(u) of
 * that filter always holds for MAXFACTOR2 >= 1).  max_factor2 = 0 is
 * nlp_predict. */
nlp_status nlp_predict_ex(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, uint32_t max_factor2,
                          float min_score, uint64_t max_edges, int repeat, nlp_edge* out, uint64_t* out_count,
                          nlp_timing* t);

/* Copy the first min(n, *count of the last prediction*) links of the last
 * nlp_predict / nlp_predict_ex / nlp_predict_device result of this handle to the
 * HOST array `out` (*copied = how many).  Valid until the next prediction on
 * the handle.  This is the second half of the count query above. */
nlp_status nlp_copy_last(nlp_graph* g, nlp_edge* out, uint64_t n, uint64_t* copied);

/* Page-locked host memory (hipHostMalloc) for result copies at the full PCIe
 * rate: the C++ header (include/nlp/predict.hxx) keeps one such staging buffer
 * per thread and converts the links from it into the reference's
 * vector<tuple> (PredictLinkResult::edges, predict.hxx:65-102). */
nlp_status nlp_host_alloc(uint64_t bytes, void** out);
void nlp_host_free(void* p);

/* Device-resident variant for a source-vertex range [u_begin, u_end) (the
 * multi-GPU shard; pass 0, UINT64_MAX for all).  `d_out` is a DEVICE array of
 * at least max_edges entries; `stream` is a hipStream_t (NULL = the graph's
 * own stream).  The call is synchronous with respect to the host: on return
 * d_out and *out_count are valid. */
nlp_status nlp_predict_device(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, float min_score,
                              uint64_t max_edges, uint64_t u_begin, uint64_t u_end, nlp_edge* d_out,
                              uint64_t* out_count, nlp_timing* t, void* stream);

/* nlp_predict_device with MAXFACTOR2 (see nlp_predict_ex). */
nlp_status nlp_predict_device_ex(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, uint32_t max_factor2,
                                 float min_score, uint64_t max_edges, uint64_t u_begin, uint64_t u_end,
                                 nlp_edge* d_out, uint64_t* out_count, nlp_timing* t, void* stream);

/* Asynchronous device prediction (serving: back-to-back calls without a host
 * wait, no counterpart in the reference).  Enqueues the same computation as
 * nlp_predict_device_ex on `stream` and returns at once when this handle's
 * last synchronous call had the same arguments and output array and ran as
 * one replayed graph (`stream` NULL = the device's default stream); otherwise
 * the call runs synchronously.  All calls of a batch use one stream.  Results (d_out of each
 * call, the last call's count and timing) are valid after nlp_sync; until then
 * the synchronous predict entry points return NLP_ERR_INVALID.  Not
 * thread-safe with other calls on the handle. */
nlp_status nlp_predict_device_async(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, uint32_t max_factor2,
                                    float min_score, uint64_t max_edges, uint64_t u_begin, uint64_t u_end,
                                    nlp_edge* d_out, void* stream);

/* Wait for the batch of nlp_predict_device_async calls: *out_count and t of
 * the last one.  NLP_ERR_RETRY when any call of the batch hit a condition the
 * synchronous path handles by redoing the call (a bucket or buffer overflow,
 * more candidate tiles than the counted passes hold).  Which call failed is
 * not known, and the calls after it ran on scratch state the failed call left
 * behind: EVERY output of the batch is invalid, and the caller redoes every
 * call of the batch with nlp_predict_device_ex.  NLP_ERR_INVALID when nothing
 * is pending. */
nlp_status nlp_sync(nlp_graph* g, uint64_t* out_count, nlp_timing* t);

/* Merge step of the multi-GPU path: given `n` device-resident edges that are the
 * concatenation, in ascending source-range order, of per-shard canonical
 * results, write the canonical global top max_edges into d_out (device).
 * Stable: equal scores keep input order, which is (u asc, v asc) across shards. */
nlp_status nlp_select_edges_device(nlp_graph* g, const nlp_edge* d_in, uint64_t n, uint64_t max_edges,
                                   nlp_edge* d_out, uint64_t* out_count, void* stream);

/* The same merge over the layout one all_gather produces (the multi-GPU
 * exchange; replaces the serial k-way heap merge of
 * predict.hxx:431-460): `nblocks` blocks of `stride` entries, block r at
 * d_blocks + r * stride holding shard r's canonical result (shards in ascending
 * source-range order).  Entry 0 of a block is its header
 * {u = count & 0xffffffff, v = count >> 32, score = bits NLP_BLOCK_MAGIC},
 * entries 1..count the result.  One pass: every entry's output position is its
 * index plus, for every other block, the number of that block's entries ranked
 * before it (binary search; ties rank lower blocks first).  Writes the
 * canonical global top max_edges into d_out.  NLP_ERR_CAPACITY when a count
 * exceeds stride - 1 or a header is malformed; *out_count then holds the
 * largest count (the caller regathers with a larger stride). */
#define NLP_BLOCK_MAGIC 0x4E4C5042u
nlp_status nlp_merge_blocks_device(nlp_graph* g, const nlp_edge* d_blocks, uint64_t stride, uint32_t nblocks,
                                   uint64_t max_edges, nlp_edge* d_out, uint64_t* out_count, void* stream);

/* Evaluation of main.cxx:48-57 on the device.  nlp_set_truth
 * keeps the directed deletions (main.cxx `deletions0`, both directions, host
 * arrays; sorted and deduplicated here) on the handle's device.
 * nlp_count_common_device counts |insertions1 ∩ deletions0| for `n` device
 * edges: both directions of every predicted link (directedInsertions,
 * main.cxx:111-119) looked up in the truth set; then precision =
 * common / (2 n) and recall = common / |deletions0| (main.cxx:199-201).
 * nlp_last_common does the same for the last prediction made on the handle. */
nlp_status nlp_set_truth(nlp_graph* g, const uint32_t* u, const uint32_t* v, uint64_t n);
nlp_status nlp_count_common_device(nlp_graph* g, const nlp_edge* d_edges, uint64_t n, uint64_t* common,
                                   void* stream);
nlp_status nlp_last_common(nlp_graph* g, uint64_t* common);

/* SURVEY §8(f) N1 on the device: the reference's ingest (main.cxx:241-245)
 * from the MatrixMarket file's directed pairs (1-based ids <= n, any order;
 * a symmetric-header file listed in both directions, as readMtxOmpW adds
 * them): every row sorted and deduplicated (readMtxOmpW), then, unless
 * `symmetric_input`, symmetrizeOmp with set_union_last_inplace's duplicate
 * rule (symmetrize.hxx:72-82, _algorithm.hxx:176-214, SURVEY A.3: a key of
 * both the row and its reverse edges is kept twice when it lies above the
 * first reverse key missing from the row), then removeSelfLoopsOmpU (one
 * (u, u) per row).  d_src / d_dst: m device ids; d_off: device array of
 * n + 2 offsets (span = n + 1, row 0 empty); d_keys: device array of
 * keys_cap entries (2 m always suffices).  *nnz = the entries;
 * NLP_ERR_INVALID (nothing written) when an id exceeds n;
 * NLP_ERR_CAPACITY (with *nnz set) when keys_cap is too small.  Ids < 2^31.
 * Synchronous; `stream` orders the work (NULL = the default stream). */
nlp_status nlp_ingest_device(const uint32_t* d_src, const uint32_t* d_dst, uint64_t m, uint64_t n,
                             int symmetric_input, uint64_t* d_off, uint32_t* d_keys, uint64_t keys_cap,
                             uint64_t* nnz, int device, void* stream);

/* SURVEY §8(f) N2 on the device: one deletion batch as main.cxx:164-169 makes
 * it -- generateEdgeDeletions(rnd, y, batch, 1, span - 1, true) (batch.hxx:
 * 29-112: per deletion up to 5 draws of u, then the floor(U deg u)-th entry of
 * N(u), both directions), tidyBatchUpdateU (keep existing, sort, unique) and
 * applyBatchUpdateOmpU (one occurrence of each deletion leaves its row).  rnd
 * is std::default_random_engine (minstd_rand0) whose state is *rng_state: pass
 * the seed for a fresh engine (default_random_engine rnd(seed)); on return it
 * holds the engine's state, so consecutive calls continue one engine like
 * main.cxx's.  The draws are made on the host (sequential by definition), the
 * entries they name, the tidy and the compaction on the device.  Inputs: the
 * CSR (d_off: span + 1, d_keys); outputs (caller's device arrays): d_off2
 * (span + 1), d_keys2 (nnz entries suffice), *nnz2, and the directed
 * deletions, sorted and unique (main.cxx `deletions0`), in d_del_u / d_del_v
 * (2 batch entries suffice), *ndel.  Synchronous. */
nlp_status nlp_delete_edges_device(const uint64_t* d_off, const uint32_t* d_keys, uint64_t span, uint64_t batch,
                                   uint32_t* rng_state, uint64_t* d_off2, uint32_t* d_keys2, uint64_t* nnz2,
                                   uint32_t* d_del_u, uint32_t* d_del_v, uint64_t* ndel, int device, void* stream);

/* The same N1 / N2 for host callers (nlp_main, C++ drivers): a device-resident
 * CSR object.  nlp_dcsr_ingest uploads the MatrixMarket file's directed pairs
 * (host arrays, as nlp::readMtxPairs returns them) and runs nlp_ingest_device;
 * nlp_dcsr_delete_batch runs nlp_delete_edges_device on it into a new object
 * and copies the directed deletions (sorted, unique; at most del_cap) to the
 * host arrays del_u / del_v (either may be NULL); nlp_graph_create_dcsr builds
 * the graph handle from it without a host round trip.  nlp_dcsr_info also
 * reports the sizes of the graph after readMtx (distinct pairs) and after
 * symmetrize (before self-loop removal), the sizes main.cxx prints
 * (main.cxx:241-245).  Synchronous; the default stream of `device`. */
typedef struct nlp_dcsr nlp_dcsr;
nlp_status nlp_dcsr_ingest(const uint32_t* src, const uint32_t* dst, uint64_t m, uint64_t n, int symmetric_input,
                           int device, nlp_dcsr** out);
nlp_status nlp_dcsr_delete_batch(const nlp_dcsr* x, uint64_t batch, uint32_t* rng_state, nlp_dcsr** out,
                                 uint32_t* del_u, uint32_t* del_v, uint64_t del_cap, uint64_t* ndel);
nlp_status nlp_dcsr_info(const nlp_dcsr* x, uint64_t* span, uint64_t* nnz, uint64_t* read_size, uint64_t* sym_size);
nlp_status nlp_dcsr_copy(const nlp_dcsr* x, uint64_t* offsets /* span + 1 */, uint32_t* keys /* nnz */);
void nlp_dcsr_destroy(nlp_dcsr* x);
nlp_status nlp_graph_create_dcsr(const nlp_dcsr* x, nlp_graph** out);

const char* nlp_status_string(nlp_status s);
const char* nlp_metric_name(nlp_metric m);

/* Library version (major*10000 + minor*100 + patch). */
int nlp_version(void);

#ifdef __cplusplus
}
#endif

#endif /* NLP_H */
