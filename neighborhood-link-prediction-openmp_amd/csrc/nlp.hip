// nlp.hip -- libnlp.so: graph handle, predict pipeline and the C-ABI of include/nlp.h.
//
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared (see build.py).  The
// product path is HIP only: there is no CPU fallback; without a gfx950 device
// every entry point returns NLP_ERR_NODEVICE.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include <new>
#include <vector>
#include <string>
#include <chrono>
#include <algorithm>
#include <thread>

#include "../../include/nlp.h"
#include "prims.hpp"
#include "kernels.hpp"
#include "lookback.hpp"
#include "group.hpp"
#include "select.hpp"
#include "sortpath.hpp"
#include "hashpath.hpp"
#include "multi.hpp"
#include "ingest.hpp"
#include "edgesort.hpp"
#include "../../include/nlp/random.hxx"

using namespace nlp;

namespace {

constexpr int GRID_CAP = 4096;  // grid-stride kernels: at most 4096 x 256 threads

inline unsigned grid_for(uint64_t n) {
  uint64_t g = (n + NT - 1) / NT;
  if (g < 1) g = 1;
  if (g > GRID_CAP) g = GRID_CAP;
  return (unsigned)g;
}

#define LAUNCH(kern, n, st, ...) hipLaunchKernelGGL(kern, dim3(grid_for(n)), dim3(NT), 0, st, __VA_ARGS__)
// one thread per item: for sparse latency-bound passes, where a grid-stride
// loop would chain several items' dependent loads in one wave
inline unsigned grid_full(uint64_t n) {
  uint64_t g = (n + NT - 1) / NT;
  return (unsigned)std::min<uint64_t>(std::max<uint64_t>(g, 1), 0x7fffffffull);
}
inline unsigned p1_grid(uint64_t S) {
  return (unsigned)std::min<uint64_t>(std::max<uint64_t>((S + P1_TILE - 1) / P1_TILE, 1), 65535);
}
#define LAUNCH_FULL(kern, n, st, ...) hipLaunchKernelGGL(kern, dim3(grid_full(n)), dim3(NT), 0, st, __VA_ARGS__)

// Buffer ids of the per-graph workspace.
enum Buf {
  B_C32, B_IOFF, B_EV, B_EU, B_EWC, B_EFIRST, B_WOFF,
  B_WKEY0, B_WKEY1, B_WVAL0, B_WVAL1, B_RFLAG, B_RID, B_RSTART,
  B_RKEY, B_RU, B_RW, B_RS, B_RFL, B_RPOS,
  B_CKEY, B_CU, B_CW, B_CS,           // candidate buffer (appended per chunk)
  B_TKEY, B_TU, B_TW, B_TS,           // compaction target
  B_TIE, B_TRANK, B_KEEP, B_KPOS,
  B_SK0, B_SK1, B_SV0, B_SV1,         // final sort
  B_HIST, B_HOFF, B_SCAN, B_SCAN2, B_SELHIST, B_SEL, B_CNT, B_EDGES,
  // v1 pipeline
  B_ARENA, B_ARENA2, B_VLIST, B_VIOFF, B_UCNT, B_UOFF, B_IEU, B_IEV, B_IEF, B_IEP, B_BUCKET,
  B_SKEY, B_SU, B_SW, B_SS, B_SFLAG, B_BIG, B_OK0, B_OK1, B_OV0, B_OV1, B_NSORT,
  B_FARENA, B_FAGG,
  // sort-grouped fast path (sortpath.hpp)
  B_SP_SURV, B_SP_RK0, B_SP_RK1, B_SP_RV0, B_SP_RV1, B_SP_STASH, B_SP_CU, B_SP_CW, B_SP_CS,
  B_SP_OK0, B_SP_OK1, B_SP_OV0, B_SP_OV1, B_SP_ARENA, B_SP_SEGCNT, B_SP_BKT,
  // hash path (hashpath.hpp)
  B_HP_WU, B_HP_FLAGS, B_HP_POS, B_HP_L0, B_HP_L1, B_HP_L2, B_HP_L3, B_HP_SMALL, B_HP_TIEK0, B_HP_TIEK1,
  B_HP_TIEI0, B_HP_TIEI1, B_EVAL, B_MKEY, B_MBND, B_HP_TIER, B_HP_SCNT, B_HP_SOFF, B_HP_SKEYS,
  B_HP_TCNT, B_HP_TPRE, B_HP_SDO, B_TSHIST, B_HH_SCAN,
  B_HB_W, B_HB_PRE, B_HB_START, B_HH_ROWS, B_HH_PRE, B_HH_MAPS, B_HH_BCNT, B_HH_BOFF, B_HH_XS, B_HH_SPRE, B_HH_SITEM, B_HH_FP, B_HH_HEAVY, B_HH_GHIST, B_HH_PART, B_HP_SE, B_HP_SR, B_HP_SMASK, B_HP_BPOS,
  B_ES_HIST, B_ES_DESC, B_ES_TMP,        // edgesort.hpp: histograms + tickets, look-back descriptors, records
  B_ES_SET, B_ES_K0, B_ES_K1,            // edgesort.hpp 8-byte keys: distinct-key set + ranks + scores, key buffers
  B_ES_CNT,                              // 8-byte keys: per-range digit counts + offsets
  B_ES_RUNS,                             // two-level order: counters, long-run and very-long-run lists
  NBUF
};

// Graph build timing (nlp_graph_build_phases): while a build runs, the time
// spent inside hipMalloc accumulates here (null: not timed).
// NLP_BUILD_TRACE=1: every such allocation (bytes, ms) on stderr (diagnostic).
thread_local double* t_alloc_ms = nullptr;
template <typename T>
hipError_t hmalloc(T** p, size_t bytes) {
  if (!t_alloc_ms) return hipMalloc((void**)p, bytes);
  const auto t0 = std::chrono::steady_clock::now();
  const hipError_t e = hipMalloc((void**)p, bytes);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *t_alloc_ms += ms;
  static const bool trace = getenv("NLP_BUILD_TRACE") && getenv("NLP_BUILD_TRACE")[0] == '1';
  if (trace) fprintf(stderr, "nlp build: hipMalloc %.3f GB %.1f ms\n", bytes / 1e9, ms);
  return e;
}

struct Workspace {
  void* p[NBUF] = {};
  size_t bytes[NBUF] = {};
  hipError_t get(int id, size_t need, void** out) {
    if (need == 0) need = 16;
    if (bytes[id] < need) {
      if (p[id]) {
        hipError_t e = hipFree(p[id]);
        if (e != hipSuccess) return e;
        p[id] = nullptr;
        bytes[id] = 0;
      }
      size_t nb = std::max(need, bytes[id] + bytes[id] / 2);
      nb = (nb + 255) & ~(size_t)255;
      hipError_t e = hmalloc(&p[id], nb);
      if (e != hipSuccess) { p[id] = nullptr; return e; }
      bytes[id] = nb;
    }
    *out = p[id];
    return hipSuccess;
  }
  void release() {
    for (int i = 0; i < NBUF; ++i) {
      if (p[i]) (void)hipFree(p[i]);
      p[i] = nullptr;
      bytes[i] = 0;
    }
  }
};

template <typename T>
hipError_t wsget(Workspace& ws, int id, uint64_t count, T** out) {
  void* p;
  hipError_t e = ws.get(id, (size_t)count * sizeof(T), &p);
  *out = (T*)p;
  return e;
}

// scan_excl_u64 over workspace scratch `id`, checked against the scratch's
// size first (round 3's C1 IHub fault was a scan of more items than its
// scratch was sized for): an undersized scratch is a sizing bug, reported as
// hipErrorInvalidValue instead of an out-of-bounds device write.
template <typename T>
hipError_t scan_ws(const Workspace& ws, int id, const T* in, uint64_t n, uint64_t* out, uint64_t* d_total,
                   hipStream_t st) {
  if (ws.bytes[id] < scan_scratch_words(n) * 8) return hipErrorInvalidValue;
  return scan_excl_u64<T>(in, n, out, d_total, (uint64_t*)ws.p[id], st);
}

}  // namespace

struct nlp_graph {
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t span = 0, nnz = 0;
  uint64_t* off = nullptr;
  uint32_t* keys = nullptr;
  uint32_t* deg = nullptr;
  uint64_t* toff = nullptr;   // transposed CSR (== off/keys when symmetric)
  uint32_t* tkeys = nullptr;
  bool symmetric = true;
  uint32_t maxdeg = 0;
  double* ctab_aa = nullptr;  // 1.0 / log((double)d), d = 0..maxdeg  (predict.hxx:788)
  double* ctab_ra = nullptr;  // 1.0 / (double)d                        (predict.hxx:828)
  uint32_t* efilt = nullptr;  // edge filter of the first-order exclusion (k_sp_runs; only without etab)
  uint32_t efbits = 0;
  uint64_t* etab = nullptr;   // exact membership table of the entries w > u (hashpath.hpp k_etab_insert)
  // the transposed sort's scratch, kept after the sort: the later build arrays (entry classes, degrees
  // and ranks, the membership table) are carved from it (gmalloc) instead of freed and re-allocated
  char* slab = nullptr;
  uint64_t slab_bytes = 0, slab_used = 0;
  uint32_t etbits = 0;
  uint64_t* host_small = nullptr;  // pinned counters
  uint64_t* host_ctr = nullptr;    // host-mapped counters written by the last kernel (sort path)
  uint64_t* host_ctr_dev = nullptr;
  uint64_t* d_sticky = nullptr;     // OR of the flags of the calls since the last async batch began
  // nlp_predict_device_async: the last synchronous call that may be replayed
  // without a wait (same arguments, first attempt, replayed graph) and the
  // batch in flight
  bool async_ok = false;
  uint64_t async_key[6] = {};  // metric | H << 32, maxf2 | min_score bits << 32, max_edges, ua, ub, (unused)
  const void* async_out = nullptr;
  int async_pending = 0;         // calls enqueued since the last nlp_sync
  bool async_last_sync = false;  // the last call of the batch ran synchronously (its results below)
  uint64_t async_count = 0;
  nlp_timing async_t{};          // the last synchronous call's timing (a replayed call's counters and
                                 // bytes are those of the eligible call, nlp_timing tmpl below)
  nlp_timing async_tmpl{};
  uint64_t async_fail = 0;       // flags of the batch's replayed calls folded in before a synchronous one
  const void* async_last_out = nullptr;
  hipStream_t async_stream = nullptr;
  hipEvent_t ev[8] = {};
  hipEvent_t gev[5] = {};  // recorded only as event nodes of captured graphs
  hipEvent_t gev_end = nullptr;  // end of a stamp-timed graph: no timestamp (NLP_END_MODE)
  int end_mode = 1;              // stamp-timed graphs end with: 0 a timing event node, 1 a no-timing event node,
                                 // 2 a no-timing event recorded on the stream after the launch
  bool last_single = false; // the last fast call replayed a single graph (timing in gev)
  Workspace ws;
  uint64_t wedge_budget = 0;
  uint64_t capE = 1u << 20, capW = 1u << 20;  // path-1 capacities (grown on overflow)
  bool force_radix = false;                    // test hook: NLP_FORCE_RADIX=1
  bool sort_grouping = true;                   // NLP_GROUPING=bucket selects the per-source bucket grouping
  bool sort_lsd = false;                       // NLP_GROUPING=lsd: full LSD record sort (no MSD buckets)
  // degree-class index (sortpath.hpp): vertices of degree 1..DCAP grouped by degree
  uint32_t* vbydeg = nullptr;
  uint64_t* sv_pack = nullptr;     // (deg v << 48 | off v) per vbydeg entry (k_sv_pack)
  uint64_t* sv_pack_in = nullptr;  // asymmetric graphs: (|I(v)| << 48 | toff v) per vbydeg entry
  std::vector<uint64_t> dstart;                // class d occupies [dstart[d], dstart[d + 1]) (class 1 at 0)
  bool use_dindex = true;                      // NLP_NO_DINDEX=1: always scan deg[] for survivors
  // the same index restricted to a source range (k_range_index; multi-GPU shards)
  uint32_t* rx_vbydeg = nullptr;               // capacity dstart[DCAP + 1], allocated once
  unsigned long long* rx_cnt = nullptr;        // DCAP + 1 class counters / cursors
  std::vector<uint64_t> rx_dstart;             // class starts of the range index
  uint64_t rx_ua = 0, rx_ub = 0;
  uint32_t rx_H = 0;                           // classes 1..rx_H built (0: none)
  bool use_rindex = true;                      // NLP_NO_RINDEX=1: ranged calls scan the full index
  // NLP_STAMP=<file>: per-workgroup phase stamps of the timed stage appended to <file> (diagnostics)
  uint64_t* d_stamp = nullptr;
  uint32_t stamp_blocks = 0;
  std::string stamp_path;
  int ex_ipt = 1;                              // k_sp_expand survivors per thread (NLP_EX_IPT: 1, 2 or 4)
  bool fuse_gather = false;                    // the last ordering pass writes the edges (NLP_FUSE_GATHER=1; measured slower)
  bool direct_emit = true;                     // count metrics: records straight into MSD buckets (NLP_DIRECT=0: off)
  bool ord11 = false;                          // fused path: three 11-bit ordering passes (NLP_ORD11=1) instead of four 8-bit
  double cp_off_w = 0;                         // wedge estimate of the last call whose counted passes overflowed
  bool counted_force = false;
  bool counted = true;                         // fused path: ordering passes 2-4 from per-tile digit counts (k_sp_cpass,
                                               // no look-back) when the candidates fit CP_MAXT tiles (NLP_COUNTED=0: off)
  bool small_order = true;                     // fused path: one launch ranks <= SO_MAX candidates
                                               // (k_sp_order_rank; NLP_SMALL_ORDER=0: off)
  double small_off_w = 0;                      // wedge estimate of the last call whose candidates did not fit it
  bool small_force = false;
  uint64_t* ord_clean = nullptr;               // the sort-path arena whose ordering descriptors are all zero
  int gr_nt = GR_NT;                           // k_sp_grouprun threads per bucket (NLP_GR_NT=512)
  bool direct_launch = false;                  // no graphs anywhere (NLP_DIRECT_LAUNCH=1)
  bool sync_direct = true;                     // stamp-timed sort path: kernels launched one by one, also for
                                               // synchronous calls (NLP_DIRECT_LAUNCH=0: one replayed hipGraph)
  bool async_direct = true;                    // asynchronous calls launched kernel by kernel (NLP_ASYNC_GRAPH=1: graphs)
  int exb_spt = 2;                             // k_sp_exbucket: survivors per thread (NLP_EXB_SPT 1, 2, 4)
  bool fuse_runs = true;                       // direct emission: grouping + scoring in one kernel (NLP_FUSE_RUNS=0: off)
  double dx_target = 256;                      // direct buckets: mean records per bucket (NLP_DX_TARGET)
  int dx_bits = 0;                             // direct buckets: forced width (NLP_DX_BITS, 0 = from dx_target)
  int hot_stage = -1;                          // sort path: stage timed as the dominant kernel (-1: the scoring
                                               // kernel k_sp_bucket / k_sp_scan<F_Runs>; NLP_HOT_STAGE)
  // co-resident workgroups of the persistent single-pass kernels (occupancy x CUs)
  unsigned occ_surv = 256, occ_exp = 256, occ_p64 = 256, occ_p32 = 256, occ_p11 = 256, occ_run = 256;
  bool split_bucket = true;                    // NLP_BUCKET_FUSED=1: score inside k_sp_bucket (one block per bucket)
  int msd_force = 0;                           // NLP_MSD_PASSES: force 1 or 2 MSD passes (tests)
  int group_sort = 2;                          // NLP_GROUP_SORT: 0 k_sp_bucket sort-only, 1 k_sp_group, 2 group only after 2 MSD passes
  uint64_t last_wedges = 0;                    // wedges of the previous fast call (sizes the MSD passes)
  double last_ok_w = 0;                        // wedge estimate of the last successful sort-path call
  bool last_ok_msd = true;                     //   and its grouping (MSD bucket passes or full LSD sort)
  int last_ok_passes = 1;
  bool use_graphs = true;                      // hipGraph replay (off with NLP_DIRECT_LAUNCH=1)
  bool graph_single = true;                    // NLP_GRAPH_SEGMENTS=1: four graph segments with host events
  uint64_t ws_gen = 0;                         // bumped whenever a workspace buffer moves
  struct Cached {
    int metric;
    uint32_t H;
    float min_score;
    uint64_t max_edges, ua, ub, capW, gen;
    uint32_t maxf2;
    int mode;  // fast-path variant (graph shapes differ)
    void* out;
    hipGraphExec_t exec[4];
    bool single;  // one graph with event-record nodes (else four segments)
    uint64_t last_use;
  };
  std::vector<Cached> graphs;
  uint64_t use_clock = 0;
  // hash path: per-workgroup global tables of bins 2 and 3 (kept clean between calls)
  uint32_t* hp_scratch = nullptr;              // k_hp_part: per-workgroup wedge scratch (w and v)
  uint32_t* tile_row = nullptr;                // row of the first entry of every HP_WTILE-entry tile
  uint8_t* dcls = nullptr;                     // min(deg keys[e], 255) per adjacency entry (path 4's survivor lists)
  uint32_t* kdeg = nullptr;                    // deg keys[e] per adjacency entry (path 4's count-metric row kernels)
  uint8_t* drank = nullptr;                    // entries with deg v <= 254: the row's rank in N(v) (survivor suffixes)
  uint32_t* xs = nullptr;                      // per row: entries of N(u) at or below u (the exclusion walks the rest)
  // class-ordered short lists (hashpath.hpp k_sl_sort): per row its entries v with 1 <= deg v <= 254 by deg v
  uint64_t* sl_off = nullptr;                  // [S + 1] row offsets
  uint32_t* sl_keys = nullptr;                 // v
  uint64_t* sl_sdo = nullptr;                  // deg v << 48 | n << 40 | o (as the survivor lists)
  uint8_t* sl_cls = nullptr;                   // deg v
  uint32_t* sl_pn = nullptr;                   // inclusive prefix of n over the row's list (W+(u) of a prefix)
  uint64_t sl_n = 0;
  uint32_t sl_cap = 0;                         // classes kept: S(u) for H <= sl_cap
  // evaluation (main.cxx:48-57): sorted directed deletion keys, and the last prediction's device output
  uint64_t* truth = nullptr;
  uint64_t ntruth = 0;
  const EdgeOut* last_out = nullptr;
  uint64_t last_n = 0;
  hipStream_t last_stream = nullptr;
  unsigned hp_gp = 0;                          // workgroups of k_hp_part
  uint64_t hp_scap = 0;                        // scratch words per workgroup and array
  uint64_t hp_min_wedges = 1ull << 26;         // NLP_HASH_MIN_WEDGES: estimated wedges above which path 4 runs
  int hash_mode = 0;                           // NLP_HASH: 0 auto, 1 always, -1 never
  // test hooks: NLP_HASH_EMIT (emission slots per chunk), NLP_HASH_MINBIN (smallest bin), NLP_HASH_SCAP
  // (scratch words per workgroup)
  uint64_t hp_emit = 0;
  int hp_minbin = 0;
  bool sv_pack_on = true;   // NLP_SV_PACK=0: survivors' rows loaded unpacked (parity of the packed loads)
  int hh_tl = 0;             // hub pass: table log for the item plan (NLP_HASH_HUB_TL, 7..13; small values test the splits)
  // survivor lists: three streaming kernels (k_dc_*; a one-pass build with a decoupled look-back measured
  // slower, 7.2 vs 5.9 ms on C4 H=16, and was removed in round 5)
  unsigned occ_es = 256;     // resident k_es_pass workgroups
  unsigned occ_hb = 512;     // resident k_hp_batch workgroups (count-metric build)
  uint64_t es_epoch = 0;     // look-back descriptor epoch of the last edgesort pass
  size_t es_desc_bytes = 0;  // descriptor buffer the epochs refer to (a new buffer restarts them)
  const void* es_desc_ptr = nullptr;  // and its address (a same-size reallocation restarts them too)
  unsigned occ_es8 = 256;    // resident workgroups of k_es_pass8
  unsigned occ_es8w = 256;   // and of its wide form (ES8_NTW threads)
  int es8_nt = ES8_NTW;      // the 8-byte passes' workgroup: ES8_NTW (8192-key tiles) or ES8_NT threads
                             // (NLP_ES8_NT=256; C4 H=16 orders: 0.3-0.6 ms faster wide)
  int es_k8 = 1;             // the final order over rank-compressed 8-byte keys when it qualifies: 1 from
                             // ES8_MIN links on, 2 always (tests), 0 never (NLP_ES8)
  int es_runs = 1;           // the 8-byte order's two-level form (passes over (rank, u), runs put in w order):
                             // 1 when it saves two passes or more, 2 whenever the 8-byte order runs, 0 never
                             // (NLP_ES_RUNS)
  uint32_t es_rs = ER_RSMAX;   // runs up to this long ranked by k_es_runs (NLP_ES_RS: small values test the rest)
  uint32_t es_lcap = EL_CAPMAX;  // long runs up to this long sorted in LDS by k_es_long (NLP_ES_LCAP)
  bool hp_aa = true;         // AA / RA route to path 4 like the count metrics (NLP_HASH_AA=0: sort paths only)
  bool hh_sort = true;       // hub pass, AA / RA: sort-mode items instead of the ordered re-walk (NLP_HASH_HUB_SORT=0)
  uint32_t hp_uxf = HB_XF;   // exclusion by the membership table for slices beyond hp_uxf x W
                             // (NLP_HASH_UX=off: always marks; =0: always the table)
  int hp_rowb = 1;           // bin 1, count metrics: tiered 256-thread rows (NLP_HASH_ROWB=0: k_hp_block;
                             // 2: every row in the 8192-entry tier, 3: none in the 2048-entry tier -- tests)
  uint32_t hh_dw = HH_DW;    // hub pass, counts: direct-counter range width (NLP_HH_DIRECT=0 off, small values test it)
  uint32_t hh_scap = HH_SCAP;  // sort-mode wedges per item (NLP_HASH_HUB_SCAP: small values test the splits and HH_BIG)
  uint64_t hh_bw = HH_BW;   // hub pass: W(u) per w-bucket (NLP_HASH_HUB_BW; large values test the sub-range passes)
  int hp_hub_min = 2;        // lowest bin the hub pass takes (NLP_HASH_HUB_MIN=1: bin 1 too)
  bool hp_hub = true;        // path 4: bins 2 / 3 by the hub pass (k_hh_*; NLP_HASH_HUB=0: k_hp_part)
  bool hp_batch = true;      // path 4: bin-0 tiers 0 / 1 in row batches (k_hp_batch; NLP_HASH_BATCH=0: a wave per row)
  // (u64, u32) sorts of paths 2 / 4 by onesweep passes (NLP_OS_SORT=1); the default hist / scan / scatter
  // passes measured faster at these sizes (C4 JAC H=16 ordering: 22 vs 77 ms; C3 AA H=16 path 2: 122 vs 418 ms)
  bool hp_dcls = true;       // survivor lists by filtering N(u) with the degree classes (NLP_HASH_DCLS=0: in-edge atomics)
  uint64_t hp_scap_force = 0;
  std::vector<uint64_t> deg_hist;              // vertices per degree 0..DCAP, for wedge estimates
  uint64_t big_deg2 = 0;                       // sum of deg^2 over vertices of degree > DCAP
  // multi-device group (nlp_graph_create_multi; SURVEY §8(b) devices[], ndev): no CSR of its own
  bool is_group = false;
  std::vector<nlp_graph*> members;             // one full graph per distinct device, members[0] on devices[0]
  std::vector<int> part_member;                // member of each logical partition p (= devices[p])
  std::vector<uint64_t> part_bounds;           // P + 1 source bounds, balanced for the hub threshold part_H
  int64_t part_H = -1;
  std::vector<EdgeOut*> part_buf;              // per partition, on its member's device: header + its list
  std::vector<uint64_t> part_cap;
  std::vector<uint64_t*> part_hist;            // per partition: first / last run bounds of 65536 key bins
  EdgeOut* gather_buf = nullptr;               // on members[0]: the partitions' shares, one block each
  uint64_t gather_cap = 0;
  EdgeOut* group_out = nullptr;                // on members[0]: the merged result of a host-output call
  uint64_t group_out_cap = 0;
  // phases of the build (nlp_graph_build_phases): name and host wall ms, the stream drained at each boundary
  std::vector<std::pair<const char*, double>> build_phases;
  double build_alloc_ms = 0;                   // of the build, the time inside hipMalloc
};

namespace {

nlp_status from_hip(hipError_t e) {
  if (e == hipSuccess) return NLP_OK;
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return NLP_ERR_NOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return NLP_ERR_NODEVICE;
  return NLP_ERR_DEVICE;
}

// debug_on() (build-time) reports the failing runtime call on stderr
inline bool debug_on() {
  constexpr bool on = false;  // a build-time switch: the failing runtime call on stderr
  return on;
}
#define TRY(x)                                                                                     \
  do {                                                                                             \
    hipError_t e__ = (x);                                                                          \
    if (e__ != hipSuccess) {                                                                       \
      if (debug_on()) fprintf(stderr, "nlp: %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e__)); \
      return from_hip(e__);                                                                        \
    }                                                                                              \
  } while (0)

// Wait for an event by polling: a blocking wait can add tens of microseconds
// of wake-up latency to every call, which is a large share of a fast prediction.
// The same for everything queued on a stream (a graph without an end event).
hipError_t wait_stream(hipStream_t st) {
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q != hipErrorNotReady) return q;
  }
}

hipError_t wait_event(hipEvent_t e) {
  for (;;) {
    const hipError_t q = hipEventQuery(e);
    if (q != hipErrorNotReady) return q;
  }
}

nlp_status check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return NLP_ERR_NODEVICE;
  if (device < 0 || device >= n) return NLP_ERR_INVALID;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return NLP_ERR_NODEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return NLP_ERR_NODEVICE;
  return NLP_OK;
}

// read `n` u64 device words into pinned host memory and wait
hipError_t read_small(nlp_graph* g, const uint64_t* d, int n, hipStream_t st) {
  hipError_t e = hipMemcpyAsync(g->host_small, d, 8 * n, hipMemcpyDeviceToHost, st);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(st);
}

// A per-graph build array carved from the slab (the transposed sort's kept
// scratch) when it fits, else its own allocation.  The driver wipes freed HBM
// asynchronously and an allocation that needs those pages waits for the wipe:
// the round-6 bench box where a box before us had freed its memory waited
// 3.4 s in the membership table's hipMalloc after the sort's scratch was
// freed (0.6 s builds elsewhere).  Carving takes no free and no allocation.
template <typename T>
hipError_t gmalloc(nlp_graph* g, T** p, size_t bytes) {
  bytes = (bytes + 255) & ~(size_t)255;
  if (g->slab && g->slab_used + bytes <= g->slab_bytes) {
    *p = (T*)(g->slab + g->slab_used);
    g->slab_used += bytes;
    return hipSuccess;
  }
  return hmalloc(p, bytes);
}
void gfree(nlp_graph* g, void* p) {
  if (!p) return;
  if (g->slab && (char*)p >= g->slab && (char*)p < g->slab + g->slab_bytes) return;  // the slab's: freed with it
  (void)hipFree(p);
}

void destroy_graph(nlp_graph* g) {
  if (!g) return;
  if (g->is_group) {
    for (size_t q = 0; q < g->part_buf.size(); ++q) {
      (void)hipSetDevice(g->members[g->part_member[q]]->device);
      if (g->part_buf[q]) (void)hipFree(g->part_buf[q]);
      if (q < g->part_hist.size() && g->part_hist[q]) (void)hipFree(g->part_hist[q]);
    }
    if (!g->members.empty()) (void)hipSetDevice(g->members[0]->device);
    if (g->gather_buf) (void)hipFree(g->gather_buf);
    if (g->group_out) (void)hipFree(g->group_out);
    for (nlp_graph* m : g->members) destroy_graph(m);
    delete g;
    return;
  }
  (void)hipSetDevice(g->device);
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  for (auto& c : g->graphs)
    for (auto& x : c.exec)
      if (x) (void)hipGraphExecDestroy(x);
  g->graphs.clear();
  if (g->d_stamp) (void)hipFree(g->d_stamp);
  if (g->hp_scratch) (void)hipFree(g->hp_scratch);
  if (g->tile_row) (void)hipFree(g->tile_row);
  gfree(g, g->dcls);
  gfree(g, g->kdeg);
  gfree(g, g->drank);
  if (g->xs) (void)hipFree(g->xs);
  for (void* p : {(void*)g->sl_off, (void*)g->sl_keys, (void*)g->sl_sdo, (void*)g->sl_cls, (void*)g->sl_pn})
    if (p) (void)hipFree(p);
  if (g->truth) (void)hipFree(g->truth);
  g->ws.release();
  if (!g->symmetric) {
    if (g->toff) (void)hipFree(g->toff);
    if (g->tkeys) (void)hipFree(g->tkeys);
  }
  if (g->off) (void)hipFree(g->off);
  if (g->keys) (void)hipFree(g->keys);
  if (g->deg) (void)hipFree(g->deg);
  if (g->vbydeg) (void)hipFree(g->vbydeg);
  if (g->sv_pack) (void)hipFree(g->sv_pack);
  if (g->sv_pack_in) (void)hipFree(g->sv_pack_in);
  if (g->ctab_aa) (void)hipFree(g->ctab_aa);
  if (g->ctab_ra) (void)hipFree(g->ctab_ra);
  if (g->efilt) (void)hipFree(g->efilt);
  gfree(g, g->etab);
  if (g->slab) (void)hipFree(g->slab);
  if (g->rx_vbydeg) (void)hipFree(g->rx_vbydeg);
  if (g->rx_cnt) (void)hipFree(g->rx_cnt);
  for (int i = 0; i < 8; ++i)
    if (g->ev[i]) (void)hipEventDestroy(g->ev[i]);
  for (int i = 0; i < 5; ++i)
    if (g->gev[i]) (void)hipEventDestroy(g->gev[i]);
  if (g->gev_end) (void)hipEventDestroy(g->gev_end);
  if (g->host_small) (void)hipHostFree(g->host_small);
  if (g->host_ctr) (void)hipHostFree(g->host_ctr);
  if (g->d_sticky) (void)hipFree(g->d_sticky);
  if (g->stream) (void)hipStreamDestroy(g->stream);
  delete g;
}

int log2_host(uint64_t x) {  // ceil(log2(x)), x >= 1
  int b = 0;
  while (b < 63 && (1ull << b) < x) ++b;
  return b;
}

int bits_for(uint64_t maxval) {  // bits needed to represent values <= maxval
  int b = 0;
  while (b < 64 && (maxval >> b)) ++b;
  return b;
}

// Class-ordered short lists (hashpath.hpp k_sl_sort): the degree-class
// compaction at H = HP_DCLS_MAX over the whole graph (k_dc_count, scan,
// k_dc_place, k_dc_gather: the rows' short entries in N(u)'s order, packed,
// with their rows), the row offsets from the per-row counts, then the stable
// per-row sort by class.  Skipped -- the calls then compact per call -- when
// the lists and their build scratch would take more than a quarter of the free
// HBM; any allocation failure also just skips them.
// Wall time of the build's phases (nlp_graph_build_phases): mark() drains the
// graph's stream and closes a phase; hipMalloc time is summed on the side.
struct BuildClock {
  nlp_graph* g;
  std::chrono::steady_clock::time_point t;
  double alloc = 0;
  double* prev;
  explicit BuildClock(nlp_graph* gr) : g(gr), t(std::chrono::steady_clock::now()), prev(t_alloc_ms) {
    g->build_phases.clear();
    t_alloc_ms = &alloc;
  }
  ~BuildClock() { t_alloc_ms = prev; }  // (g may be gone: an error path destroys it first)
  hipError_t mark(const char* name) {
    const hipError_t e = hipStreamSynchronize(g->stream);
    const auto n = std::chrono::steady_clock::now();
    g->build_phases.emplace_back(name, std::chrono::duration<double, std::milli>(n - t).count());
    g->build_alloc_ms = alloc;
    t = n;
    return e;
  }
};

template <typename T>
bool dmalloc(T** out, uint64_t n) {  // device allocation of n items; a failure is cleared and reported as false
  void* x = nullptr;
  if (hmalloc(&x, std::max<uint64_t>(n, 1) * sizeof(T)) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return false;
  }
  *out = (T*)x;
  return true;
}

struct DevTemps {  // device scratch freed on scope exit
  std::vector<void*> p;
  ~DevTemps() {
    for (void* x : p) (void)hipFree(x);
  }
  template <typename T>
  bool get(T** out, uint64_t n) {
    if (!dmalloc(out, n)) return false;
    p.push_back(*out);
    return true;
  }
};

nlp_status build_short_lists(nlp_graph* g, uint32_t cap) {
  hipStream_t st = g->stream;
  const uint64_t S = g->span, M = g->nnz;
  const uint64_t nt = (M + HP_WTILE - 1) / HP_WTILE;
  DevTemps tmp;
  uint32_t* tcn;
  uint64_t *tpre, *scr;
  uint8_t* smask;
  if (!tmp.get(&tcn, nt) || !tmp.get(&tpre, nt + 1) || !tmp.get(&smask, nt * 64) ||
      !tmp.get(&scr, scan_scratch_words(std::max(nt, S)) + 16))
    return NLP_OK;
  const unsigned gt = (unsigned)std::min<uint64_t>((nt + NWAVE - 1) / NWAVE, 16384);
  size_t fr = 0, tot = 0;
  TRY(hipMemGetInfo(&fr, &tot));
  fr += g->slab ? g->slab_bytes - g->slab_used : 0;  // the slab's rest: free HBM before the slab was kept
  // the classes kept: up to HP_DCLS_MAX, fewer (128, 64, 32, 16) while the lists and their build would take more
  // than a quarter of the free HBM (peak 29 B per short entry + 20 B per row; kept 17 B + 8 B)
  uint64_t L = 0;
  for (;;) {
    hipLaunchKernelGGL(k_dc_count, dim3(gt), dim3(NT), 0, st, (const uint8_t*)g->dcls, cap, 0ull, M, tcn, smask);
    TRY(hipGetLastError());
    TRY(scan_excl_u64<uint32_t>(tcn, nt, tpre, tpre + nt, scr, st));
    TRY(hipMemcpyAsync(&L, tpre + nt, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    if (debug_on()) fprintf(stderr, "nlp: short lists: classes <= %u: %llu entries, %zu bytes free\n", cap,
                            (unsigned long long)L, fr);
    if (L == 0) return NLP_OK;
    if (29 * L + 20 * S <= fr / 4) break;
    if (cap <= 16) return NLP_OK;
    cap = cap > 128 ? 128 : cap / 2;
  }
  uint64_t* se;
  uint32_t *sr, *tkeys, *scnt;
  uint64_t* tsdo;
  unsigned long long* wu;
  if (!tmp.get(&se, L) || !tmp.get(&sr, L) || !tmp.get(&tkeys, L) || !tmp.get(&tsdo, L) || !tmp.get(&wu, S) ||
      !tmp.get(&scnt, S))
    return NLP_OK;
  GraphView gv0{};
  gv0.off = g->off;
  gv0.keys = g->keys;
  gv0.deg = g->deg;
  TRY(hipMemsetAsync(wu, 0, S * 8, st));
  hipLaunchKernelGGL(k_dc_place, dim3(gt), dim3(NT), 0, st, gv0, (const uint8_t*)smask, 0ull, S, 0ull, M,
                     (const uint32_t*)g->tile_row, (const uint64_t*)tpre, se, sr);
  hipLaunchKernelGGL(k_dc_gather, dim3((unsigned)std::min<uint64_t>((L + NT - 1) / NT, 65536)), dim3(NT), 0, st, gv0,
                     (const uint8_t*)g->dcls, (const uint8_t*)g->drank, (const uint64_t*)se, (const uint32_t*)sr, L,
                     tkeys, tsdo, wu);
  TRY(hipGetLastError());
  LAUNCH(k_hp_unpack, S, st, wu, scnt, S);
  TRY(hipGetLastError());
  TRY(hipStreamSynchronize(st));
  for (void* x : {(void*)se, (void*)sr}) {  // entries and rows are done with: room for the sorted copy
    (void)hipFree(x);
    tmp.p.erase(std::find(tmp.p.begin(), tmp.p.end(), x));
  }
  nlp_graph& G = *g;
  if (!dmalloc(&G.sl_off, S + 1) || !dmalloc(&G.sl_keys, L) || !dmalloc(&G.sl_sdo, L) || !dmalloc(&G.sl_cls, L) ||
      !dmalloc(&G.sl_pn, L)) {
    for (void* p : {(void*)G.sl_off, (void*)G.sl_keys, (void*)G.sl_sdo, (void*)G.sl_cls, (void*)G.sl_pn})
      if (p) (void)hipFree(p);
    G.sl_off = nullptr;
    G.sl_keys = nullptr;
    G.sl_sdo = nullptr;
    G.sl_cls = nullptr;
    G.sl_pn = nullptr;
    return NLP_OK;
  }
  TRY(scan_excl_u64<uint32_t>(scnt, S, G.sl_off, G.sl_off + S, scr, st));
  // rows of SL_LONG short entries or more (hubs) are sorted by a workgroup each
  uint32_t *lrows = nullptr, *nlong = nullptr;
  const bool lr_ok = tmp.get(&lrows, L / SL_LONG + 1) && tmp.get(&nlong, 1);
  if (lr_ok) TRY(hipMemsetAsync(nlong, 0, 4, st));
  hipLaunchKernelGGL(k_sl_sort, dim3((unsigned)std::min<uint64_t>((S + NWAVE - 1) / NWAVE, 65536)), dim3(NT), 0, st,
                     (const uint64_t*)G.sl_off, S, (const uint32_t*)tkeys, (const uint64_t*)tsdo, G.sl_keys, G.sl_sdo,
                     G.sl_cls, G.sl_pn, lr_ok ? (uint64_t)SL_LONG : ~0ull, lrows, nlong);
  TRY(hipGetLastError());
  uint32_t nl = 0;
  if (lr_ok) {
    TRY(hipMemcpyAsync(&nl, nlong, 4, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
  }
  if (nl)
    hipLaunchKernelGGL(k_sl_sort_long, dim3(std::min<uint32_t>(nl, 65535u)), dim3(SLL_NT), 0, st,
                       (const uint64_t*)G.sl_off, (const uint32_t*)lrows, nl, (const uint32_t*)tkeys,
                       (const uint64_t*)tsdo, G.sl_keys, G.sl_sdo, G.sl_cls, G.sl_pn);
  TRY(hipGetLastError());
  TRY(hipStreamSynchronize(st));
  G.sl_n = L;
  G.sl_cap = cap;
  return NLP_OK;
}

// The 8-byte passes' launch shape: threads per workgroup, keys per tile,
// resident workgroups (NLP_ES8_NT=512: the wide form).
struct Es8Shape {
  int nt;
  uint64_t tile;
  unsigned occ;
};
Es8Shape es8_shape(const nlp_graph* g) {
  return g->es8_nt == ES8_NTW ? Es8Shape{ES8_NTW, (uint64_t)ES8_NTW * ES8_IPT, g->occ_es8w}
                              : Es8Shape{ES8_NT, (uint64_t)ES8_NT * ES8_IPT, g->occ_es8};
}
void es8_pass(const Es8Shape& sh8, bool last, uint32_t G, hipStream_t st, const float* rscore, const uint64_t* src,
              uint64_t* dst, EdgeOut* out, uint64_t n, int vb, int shift, const uint32_t* offs, uint32_t tpw,
              uint64_t nout) {
  if (sh8.nt == ES8_NTW) {
    if (last) hipLaunchKernelGGL((k_es_pass8<true, ES8_NTW>), dim3(G), dim3(ES8_NTW), 0, st, rscore, src, dst, out, n, vb, shift, offs, tpw, G, nout);
    else hipLaunchKernelGGL((k_es_pass8<false, ES8_NTW>), dim3(G), dim3(ES8_NTW), 0, st, rscore, src, dst, out, n, vb, shift, offs, tpw, G, nout);
  } else {
    if (last) hipLaunchKernelGGL((k_es_pass8<true>), dim3(G), dim3(ES8_NT), 0, st, rscore, src, dst, out, n, vb, shift, offs, tpw, G, nout);
    else hipLaunchKernelGGL((k_es_pass8<false>), dim3(G), dim3(ES8_NT), 0, st, rscore, src, dst, out, n, vb, shift, offs, tpw, G, nout);
  }
}

// A stable LSD sort of n 8-byte keys on the 8-bit digits at `shifts` with
// the order's range-local passes (edgesort.hpp k_es_cnt8 / k_es_off8 /
// k_es_pass8: a workgroup per range of consecutive tiles, digit runs written
// to the range's running offsets): the graph build's transposed sort.
// *which = 1: the result is in k1.  *done = false (nothing sorted) when n needs
// more than the passes' 32-bit offsets.
nlp_status lsd8_keys(nlp_graph* g, uint64_t* k0, uint64_t* k1, uint64_t n, const int* shifts, int np, int* which,
                     hipStream_t st, bool* done) {
  *done = false;
  *which = 0;
  if (n == 0 || n >= (1ull << 32) || np > ES_MAXP) return NLP_OK;
  Workspace& ws = g->ws;
  const Es8Shape sh8 = es8_shape(g);
  const uint64_t ntiles = (n + sh8.tile - 1) / sh8.tile;
  uint32_t G = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({ntiles, (uint64_t)sh8.occ, (uint64_t)ES8_GMAX}));
  const uint32_t tpw = (uint32_t)((ntiles + G - 1) / G);
  G = (uint32_t)((ntiles + tpw - 1) / tpw);  // every range non-empty
  uint32_t* hw;  // [np][256] digit totals
  TRY(wsget(ws, B_ES_HIST, (uint64_t)ES_MAXP * 256 + ES_MAXP + 4, &hw));
  TRY(hipMemsetAsync(hw, 0, (uint64_t)np * 256 * 4, st));
  uint32_t* cnt;  // [256][G] range counts, then [256][G] offsets
  TRY(wsget(ws, B_ES_CNT, (uint64_t)2 * 256 * G, &cnt));
  uint32_t* offs = cnt + (uint64_t)256 * G;
  const uint64_t* src = k0;
  for (int r = 0; r < np; ++r) {
    uint64_t* dst = (r & 1) ? k0 : k1;
    hipLaunchKernelGGL(k_es_cnt8, dim3(G), dim3(ES_NT), 0, st, src, n, shifts[r], cnt, hw + r * 256, tpw, G,
                       sh8.tile);
    hipLaunchKernelGGL(k_es_off8, dim3(256), dim3(ES8_GMAX), 0, st, (const uint32_t*)cnt,
                       (const uint32_t*)(hw + r * 256), G, offs);
    es8_pass(sh8, false, G, st, nullptr, src, dst, nullptr, n, 0, shifts[r], offs, tpw, 0);
    TRY(hipGetLastError());
    src = dst;
  }
  *which = np & 1;
  *done = true;
  return NLP_OK;
}

// Build everything derived from off/keys (already on the device).
nlp_status finish_graph(nlp_graph* g, BuildClock& clk) {
  hipStream_t st = g->stream;
  const uint64_t S = g->span, M = g->nnz;
  uint32_t* flags;  // [0] bad, [1] maxdeg, [2] asym
  TRY(wsget(g->ws, B_CNT, 8, &flags));
  TRY(hipMemsetAsync(flags, 0, 32, st));
  TRY(hmalloc(&g->deg, std::max<uint64_t>(S, 1) * 4));
  LAUNCH(k_degrees, S, st, g->off, S, g->deg, flags + 1, flags);
  TRY(hipGetLastError());
  unsigned long long* desc = (unsigned long long*)(flags + 4);  // [0] all descents, [1] at row starts
  if (M) {
    LAUNCH(k_check_keys, M, st, g->keys, S, M, flags, desc);
    LAUNCH(k_row_descents, S, st, g->off, g->keys, S, M, desc);
    TRY(hipGetLastError());
  }
  TRY(hipMemcpyAsync(g->host_small, flags, 32, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  uint32_t hf[8];
  memcpy(hf, g->host_small, 32);
  uint64_t hd[2];
  memcpy(hd, hf + 4, 16);
  if (hf[0] || hd[0] != hd[1]) return NLP_ERR_INVALID;
  g->maxdeg = hf[1];
  // the offsets must also start at 0 and end at nnz
  uint64_t ends[2];
  TRY(hipMemcpy(&ends[0], g->off, 8, hipMemcpyDeviceToHost));
  TRY(hipMemcpy(&ends[1], g->off + S, 8, hipMemcpyDeviceToHost));
  if (ends[0] != 0 || ends[1] != M) return NLP_ERR_INVALID;
  TRY(clk.mark("degrees"));
  // per row the entries of N(u) at or below u: the first-order exclusion only
  // marks x > u (predict.hxx:306-307 zeroes all of N(u), but only w > u are
  // candidates), so path 4's row kernels walk N(u) from there
  if (S > 0 && !(getenv("NLP_HASH_XS") && getenv("NLP_HASH_XS")[0] == '0')) {
    if (hmalloc(&g->xs, S * 4) == hipSuccess) {
      LAUNCH(k_hp_xs, S, st, (const uint64_t*)g->off, (const uint32_t*)g->keys, S, g->xs);
      TRY(hipGetLastError());
    } else {
      (void)hipGetLastError();
      g->xs = nullptr;
    }
  }
  // row of every HP_WTILE-entry adjacency tile (path 4's edge-parallel work estimate)
  TRY(hmalloc(&g->tile_row, (M / HP_WTILE + 2) * 4));
  TRY(hipMemsetAsync(g->tile_row, 0, (M / HP_WTILE + 2) * 4, st));
  LAUNCH(k_hp_tile_rows, S, st, (const uint64_t*)g->off, S, g->tile_row);
  TRY(hipGetLastError());
  TRY(clk.mark("row_index"));

  // Transposed adjacency I(v): stable radix sort of (v << 32 | u).
  g->symmetric = true;
  g->toff = g->off;
  g->tkeys = g->keys;
  if (M) {
    uint64_t *k0, *k1, *scan, *hoff;
    uint32_t* hist;
    TRY(hmalloc(&g->slab, 2 * M * 8));  // the sort's two key buffers, kept for the later arrays
    g->slab_bytes = 2 * M * 8;
    g->slab_used = 0;
    k0 = (uint64_t*)g->slab;
    k1 = k0 + M;
    uint64_t* toff;
    uint32_t* tkeys;
    TRY(hmalloc(&toff, (S + 1) * 8));
    TRY(hmalloc(&tkeys, M * 4));
    const unsigned gk = (unsigned)std::min<uint64_t>((M / HP_WTILE + NWAVE) / NWAVE + 1, 65536);
    hipLaunchKernelGGL(k_transpose_keys, dim3(gk), dim3(NT), 0, st, (const uint64_t*)g->off, (const uint32_t*)g->keys,
                       S, M, (const uint32_t*)g->tile_row, k0);
    TRY(hipGetLastError());
    // the keys come in CSR order (u ascending), so a stable sort on the v bytes
    // alone leaves every I(v) sorted by u: half the passes of a full key sort
    int vb = bits_for(S - 1);
    int shifts[4], np = 0;
    for (int b = 0; b < vb; b += 8) shifts[np++] = 32 + b;       // v bytes (high word)
    int which = 0;
    bool sorted = false;
    const char* tl = getenv("NLP_TRANSPOSE_LSD8");
    if (!(tl && tl[0] == '0')) {
      nlp_status s8 = lsd8_keys(g, k0, k1, M, shifts, np, &which, st, &sorted);
      if (s8 != NLP_OK) return s8;
    }
    if (!sorted) {  // beyond 2^32 entries: the general sort
      uint64_t nb = rs_blocks(M);
      TRY(wsget(g->ws, B_HIST, RS_BINS * nb, &hist));
      TRY(wsget(g->ws, B_HOFF, RS_BINS * nb, &hoff));
      TRY(wsget(g->ws, B_SCAN, scan_scratch_words(RS_BINS * nb) + 16, &scan));
      SortScratch sc{hist, hoff, scan, nb};
      TRY(sort_pairs_u64(k0, nullptr, k1, nullptr, M, shifts, np, sc, &which, st));
    }
    LAUNCH(k_toff_split, M + 1, st, (const uint64_t*)(which ? k1 : k0), M, S, toff, tkeys);
    TRY(hipGetLastError());
    LAUNCH(k_diff_u64, S + 1, st, toff, g->off, S + 1, flags + 2);
    LAUNCH(k_diff_u32, M, st, tkeys, g->keys, M, flags + 2);
    TRY(hipGetLastError());
    TRY(hipMemcpyAsync(g->host_small, flags + 2, 4, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    uint32_t asym;
    memcpy(&asym, g->host_small, 4);
    if (asym) {
      g->symmetric = false;
      g->toff = toff;
      g->tkeys = tkeys;
    } else {
      TRY(hipFree(toff));
      TRY(hipFree(tkeys));
    }
  }
  // the sort's other scratch goes back; its key buffers (2 x 8 B per entry)
  // stay as the slab the later arrays are carved from (gmalloc)
  g->ws.release();
  TRY(clk.mark("transpose"));
  // Degree-class index: survivors of any H <= DCAP without a pass over deg[].
  {
    uint32_t* hist;
    TRY(wsget(g->ws, B_C32, DCAP + 2, &hist));
    TRY(hipMemsetAsync(hist, 0, (DCAP + 2) * 4, st));
    hipLaunchKernelGGL(k_deg_class_hist, dim3(grid_for(S)), dim3(NT), 0, st, (const uint32_t*)g->deg, S, hist);
    TRY(hipGetLastError());
    std::vector<uint32_t> hh(DCAP + 2);
    TRY(hipMemcpyAsync(hh.data(), hist, (DCAP + 2) * 4, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    g->deg_hist.assign(hh.begin(), hh.end());
    g->deg_hist.resize(DCAP + 1);  // degrees 0..DCAP; above DCAP: big_deg2
    {
      unsigned long long* d2;
      TRY(wsget(g->ws, B_HP_SMALL, 8, &d2));
      TRY(hipMemsetAsync(d2, 0, 8, st));
      hipLaunchKernelGGL(k_sum_deg2_above, dim3(grid_for(S)), dim3(NT), 0, st, (const uint32_t*)g->deg, S, DCAP, d2);
      TRY(hipGetLastError());
      TRY(hipMemcpyAsync(&g->big_deg2, d2, 8, hipMemcpyDeviceToHost, st));
      TRY(hipStreamSynchronize(st));
    }
    g->dstart.assign(DCAP + 2, 0);
    for (uint32_t d = 1; d <= DCAP; ++d) g->dstart[d + 1] = g->dstart[d] + hh[d];
    const uint64_t nv = g->dstart[DCAP + 1];
    TRY(hmalloc(&g->vbydeg, std::max<uint64_t>(nv, 1) * 4));
    unsigned long long* cur;
    TRY(wsget(g->ws, B_SCAN, DCAP + 2, &cur));
    TRY(hipMemcpyAsync(cur, g->dstart.data(), (DCAP + 2) * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_deg_class_scatter, dim3(grid_for(S)), dim3(NT), 0, st, (const uint32_t*)g->deg, S, cur,
                       g->vbydeg);
    TRY(hipGetLastError());
    if (const char* sp = getenv("NLP_SV_PACK")) g->sv_pack_on = sp[0] != '0';
    if (nv > 0 && g->nnz < (1ull << SV_PACK_SHIFT) && g->sv_pack_on) {
      TRY(hmalloc(&g->sv_pack, nv * 8));
      uint32_t* flag = nullptr;
      if (!g->symmetric) {
        TRY(hmalloc(&g->sv_pack_in, nv * 8));
        TRY(wsget(g->ws, B_HP_SMALL, 8, &flag));
        TRY(hipMemsetAsync(flag, 0, 4, st));
      }
      hipLaunchKernelGGL(k_sv_pack, dim3(grid_for(nv)), dim3(NT), 0, st, (const uint32_t*)g->vbydeg, nv,
                         (const uint64_t*)g->off, (const uint32_t*)g->deg, g->sv_pack, (const uint64_t*)g->toff,
                         g->sv_pack_in, flag);
      TRY(hipGetLastError());
      if (flag) {
        uint32_t hf = 0;
        TRY(hipMemcpyAsync(&hf, flag, 4, hipMemcpyDeviceToHost, st));
        TRY(hipStreamSynchronize(st));
        if (hf) {  // an in-degree beyond the pack's 16 bits: the unpacked loads
          (void)hipFree(g->sv_pack);
          (void)hipFree(g->sv_pack_in);
          g->sv_pack = g->sv_pack_in = nullptr;
        }
      }
    }
    TRY(hipStreamSynchronize(st));
  }
  TRY(clk.mark("degree_class_index"));
  // degree class of every adjacency entry (path 4 filters N(u) by it: coalesced
  // bytes instead of a degree gather per entry, to build the survivor lists
  // S(u)), the entry degrees (the count-metric row kernels carry deg w in their
  // tables) and the rank of every short-list entry's row in the list: one pass,
  // k_hp_entry_classes
  const char* hdc = getenv("NLP_HASH_DCLS");
  if (M > 0 && !(hdc && hdc[0] == '0') && g->maxdeg < (1u << 24)) {
    if (gmalloc(g, &g->dcls, M) == hipSuccess) {
      const char* hkd = getenv("NLP_HASH_KDEG");
      if (!(hkd && hkd[0] == '0') && gmalloc(g, &g->kdeg, M * 4) != hipSuccess) {
        (void)hipGetLastError();
        g->kdeg = nullptr;
      }
      const char* hdr = getenv("NLP_HASH_DRANK");
      if (!(hdr && hdr[0] == '0') && gmalloc(g, &g->drank, M) != hipSuccess) {
        (void)hipGetLastError();
        g->drank = nullptr;
      }
      const unsigned gd = (unsigned)std::min<uint64_t>((M / HP_WTILE + NWAVE) / NWAVE + 1, 65536);
      hipLaunchKernelGGL(k_hp_entry_classes, dim3(gd), dim3(NT), 0, st, (const uint64_t*)g->off,
                         (const uint32_t*)g->keys, S, M, (const uint32_t*)g->tile_row, g->dcls, g->kdeg, g->drank);
      TRY(hipGetLastError());
    } else {
      (void)hipGetLastError();
      g->dcls = nullptr;
    }
  }
  TRY(clk.mark("entry_classes"));
  {  // class-ordered short lists (the count metrics' S(u) as row prefixes; NLP_HASH_SLIST=0: per-call
     // compaction, =c: classes up to c at most)
    const char* sl = getenv("NLP_HASH_SLIST");
    const uint32_t cap = sl ? (uint32_t)std::min<long>(std::max<long>(atol(sl), 0), HP_DCLS_MAX) : HP_DCLS_MAX;
    if (g->dcls && g->drank && M > 0 && M < (1ull << HP_SDO_SH) && cap > 0) {
      nlp_status s1 = build_short_lists(g, cap);
      if (s1 != NLP_OK) return s1;
    }
  }
  TRY(clk.mark("short_lists"));
  // Exact membership table of the entries w > u for the first-order exclusion
  // (kernels.hpp et_has): one 64-byte bucket read per candidate instead of a
  // search of N(u).  At most half full; skipped (NLP_ETAB=0, or when it would
  // take more than a quarter of the free HBM) in favour of the edge filter.
  {
    const char* et = getenv("NLP_ETAB");
    if (M > 0 && !(et && et[0] == '0')) {
      unsigned long long* cnt;
      TRY(wsget(g->ws, B_HP_SMALL, 8, &cnt));
      TRY(hipMemsetAsync(cnt, 0, 8, st));
      if (g->xs) {  // the entries w > u: sum of deg u - xs[u]
        LAUNCH(k_etab_upper, S, st, (const uint32_t*)g->deg, (const uint32_t*)g->xs, S, cnt);
      } else {  // an upper bound: every entry
        TRY(hipMemcpyAsync(cnt, &M, 8, hipMemcpyHostToDevice, st));
      }
      TRY(hipGetLastError());
      uint64_t upper = 0;
      TRY(hipMemcpyAsync(&upper, cnt, 8, hipMemcpyDeviceToHost, st));
      TRY(hipStreamSynchronize(st));
      uint32_t bits = 4;
      while (bits < 40 && (1ull << bits) * ET_SLOTS < 2 * upper) ++bits;  // load <= 1/2
      const uint64_t bytes = (1ull << bits) * ET_SLOTS * 8;
      size_t fr = 0, tot = 0;
      TRY(hipMemGetInfo(&fr, &tot));
      const bool in_slab = g->slab && g->slab_used + bytes <= g->slab_bytes;
      if (upper > 0 && (in_slab || bytes < fr / 4)) {
        TRY(gmalloc(g, &g->etab, bytes));
        TRY(hipMemsetAsync(g->etab, 0xff, bytes, st));
        const unsigned gi = (unsigned)std::min<uint64_t>((M / HP_WTILE + NWAVE) / NWAVE + 1, 65536);
        hipLaunchKernelGGL(k_etab_insert, dim3(gi), dim3(NT), 0, st, (const uint64_t*)g->off,
                           (const uint32_t*)g->keys, S, M, (const uint32_t*)g->tile_row, g->etab, bits);
        TRY(hipGetLastError());
        g->etbits = bits;
      }
    }
  }
  if (g->slab && g->slab_used == 0) {  // nothing carved (no entry classes, no table): the slab goes back
    TRY(hipFree(g->slab));
    g->slab = nullptr;
    g->slab_bytes = 0;
  }
  TRY(clk.mark("membership_table"));
  // Edge filter for the first-order exclusion of the scoring kernel when there
  // is no table: one bit per (u, w) hash slot, 16 slots per adjacency entry
  // (~6 % of non-edges hit a set bit and are searched; every edge is).
  // NLP_EDGE_FILTER=0 disables it.
  {
    const char* ef = getenv("NLP_EDGE_FILTER");
    const bool both = ef && ef[0] == '2';  // also in front of the table (8 slots per entry, ~128 MB on C2)
    if (M > 0 && (!g->etab || both) && !(ef && ef[0] == '0')) {
      uint32_t bits = 20;
      while (bits < 33 && (1ull << bits) < (both ? 8 : 16) * M) ++bits;
      size_t fr = 0, tot = 0;
      TRY(hipMemGetInfo(&fr, &tot));
      if ((1ull << bits) / 8 < fr / 16) {
        TRY(hmalloc(&g->efilt, (1ull << bits) / 8));
        TRY(hipMemsetAsync(g->efilt, 0, (1ull << bits) / 8, st));
        hipLaunchKernelGGL(k_edge_filter, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, st, (const uint64_t*)g->off,
                           (const uint32_t*)g->keys, S, g->efilt, bits);
        TRY(hipGetLastError());
        g->efbits = bits;
      }
    }
  }
  TRY(clk.mark("edge_filter"));
  // AA / RA contribution tables, computed on the host with the same libm the
  // reference uses (glibc log), indexed by degree: every degree below CT_DENSE,
  // above it only the degrees some vertex has (C4: maxdeg ~5.7e6, a few
  // thousand distinct degrees above 65536), scattered on the device
  {
    constexpr uint64_t CT_DENSE = 65536;
    const uint64_t nd = (uint64_t)g->maxdeg + 1, dense = std::min(nd, CT_DENSE);
    TRY(hmalloc(&g->ctab_aa, nd * 8));
    TRY(hmalloc(&g->ctab_ra, nd * 8));
    std::vector<double> aa(dense), ra(dense);
    for (uint64_t d = 0; d < dense; ++d) {
      aa[d] = 1.0 / log((double)d);
      ra[d] = 1.0 / (double)d;
    }
    TRY(hipMemcpyAsync(g->ctab_aa, aa.data(), dense * 8, hipMemcpyHostToDevice, st));
    TRY(hipMemcpyAsync(g->ctab_ra, ra.data(), dense * 8, hipMemcpyHostToDevice, st));
    if (nd > dense) {
      const uint64_t words = (nd + 63) / 64;
      unsigned long long* pres;
      TRY(wsget(g->ws, B_C32, words * 2, (uint32_t**)&pres));
      TRY(hipMemsetAsync(pres, 0, words * 8, st));
      LAUNCH(k_deg_present, S, st, (const uint32_t*)g->deg, S, (uint32_t)dense, pres);
      TRY(hipGetLastError());
      std::vector<unsigned long long> hp(words);
      TRY(hipMemcpyAsync(hp.data(), pres, words * 8, hipMemcpyDeviceToHost, st));
      TRY(hipStreamSynchronize(st));
      std::vector<uint32_t> ds;
      std::vector<double> va, vr;
      for (uint64_t w = dense / 64; w < words; ++w)
        for (unsigned long long x = hp[w]; x; x &= x - 1) {
          const uint64_t d = w * 64 + (uint64_t)__builtin_ctzll(x);
          if (d < dense || d >= nd) continue;
          ds.push_back((uint32_t)d);
          va.push_back(1.0 / log((double)d));
          vr.push_back(1.0 / (double)d);
        }
      if (!ds.empty()) {
        uint32_t* dd;
        double *da, *dr;
        TRY(wsget(g->ws, B_HIST, ds.size(), &dd));
        TRY(wsget(g->ws, B_HOFF, ds.size(), (uint64_t**)&da));
        TRY(wsget(g->ws, B_SCAN, ds.size(), (uint64_t**)&dr));
        TRY(hipMemcpyAsync(dd, ds.data(), ds.size() * 4, hipMemcpyHostToDevice, st));
        TRY(hipMemcpyAsync(da, va.data(), va.size() * 8, hipMemcpyHostToDevice, st));
        TRY(hipMemcpyAsync(dr, vr.data(), vr.size() * 8, hipMemcpyHostToDevice, st));
        LAUNCH(k_ctab_scatter, ds.size(), st, (const uint32_t*)dd, (const double*)da, (const double*)dr,
               (uint64_t)ds.size(), g->ctab_aa, g->ctab_ra);
        TRY(hipGetLastError());
      }
    }
    TRY(hipStreamSynchronize(st));
  }
  // Wedge budget per chunk of path 2 / limit of path 1: ~1/8 of free HBM at
  // ~44 B per wedge of working set.
  size_t fr = 0, tot = 0;
  TRY(hipMemGetInfo(&fr, &tot));
  uint64_t b = (uint64_t)(fr / 8 / 44);
  g->wedge_budget = std::max<uint64_t>(1u << 20, std::min<uint64_t>(b, 1ull << 30));
  if (const char* fr = getenv("NLP_FORCE_RADIX")) g->force_radix = fr[0] == '1';
  // test hook: NLP_WEDGE_BUDGET forces path-2 chunking on small graphs
  if (const char* ev = getenv("NLP_WEDGE_BUDGET")) {
    unsigned long long v = strtoull(ev, nullptr, 10);
    if (v > 0) g->wedge_budget = v;
  }
  if (const char* de = getenv("NLP_DIRECT")) g->direct_emit = de[0] != '0';
  if (const char* dl = getenv("NLP_DIRECT_LAUNCH")) {
    g->direct_launch = dl[0] == '1';
    g->sync_direct = dl[0] != '0';
    if (g->direct_launch) g->use_graphs = false;
  }
  if (const char* cp = getenv("NLP_COUNTED")) {  // 0: off, 2: whatever the estimate (tests the F_CPASS redo)
    g->counted = cp[0] != '0';
    g->counted_force = cp[0] == '2';
  }
  if (const char* so = getenv("NLP_SMALL_ORDER")) {  // 0: off, 2: whatever the estimate (tests the F_SMALL redo)
    g->small_order = so[0] != '0';
    g->small_force = so[0] == '2';
  }
  if (const char* dbs = getenv("NLP_DX_BITS")) g->dx_bits = std::max(0, atoi(dbs));
  if (const char* sp = getenv("NLP_STAMP")) {
    g->stamp_path = sp;
    TRY(hipMalloc(&g->d_stamp, 8 * 65536 * 8));
    TRY(hipMemset(g->d_stamp, 0, 8 * 65536 * 8));
  }
  if (const char* nd = getenv("NLP_NO_DINDEX")) g->use_dindex = nd[0] != '1';
  if (const char* hm = getenv("NLP_HASH")) g->hash_mode = hm[0] == '1' ? 1 : (hm[0] == '0' ? -1 : 0);
  if (const char* hw = getenv("NLP_HASH_MIN_WEDGES")) g->hp_min_wedges = strtoull(hw, nullptr, 10);
  if (const char* he = getenv("NLP_HASH_EMIT")) g->hp_emit = strtoull(he, nullptr, 10);
  if (const char* hb = getenv("NLP_HASH_MINBIN")) g->hp_minbin = std::min(3, std::max(0, atoi(hb)));
  if (const char* hc = getenv("NLP_HASH_SCAP")) g->hp_scap_force = std::max<uint64_t>(64, strtoull(hc, nullptr, 10));
  if (const char* hd = getenv("NLP_HASH_DCLS")) g->hp_dcls = hd[0] != '0';
  if (const char* hb = getenv("NLP_HASH_BATCH")) g->hp_batch = hb[0] != '0';
  if (const char* hh = getenv("NLP_HASH_HUB")) g->hp_hub = hh[0] != '0';
  if (const char* hm = getenv("NLP_HASH_HUB_MIN")) g->hp_hub_min = std::max(1, std::min(2, atoi(hm)));
  if (const char* hw = getenv("NLP_HASH_HUB_BW")) g->hh_bw = std::max<uint64_t>(64, strtoull(hw, nullptr, 10));
  if (const char* ht = getenv("NLP_HASH_HUB_TL")) g->hh_tl = std::max(7, std::min(HH_TL, atoi(ht)));
  if (const char* hs = getenv("NLP_HASH_HUB_SORT")) g->hh_sort = hs[0] != '0';
  if (const char* hr = getenv("NLP_HASH_ROWB")) g->hp_rowb = atoi(hr);
  if (const char* e8 = getenv("NLP_ES8")) g->es_k8 = std::min(2, std::max(0, atoi(e8)));
  if (const char* en = getenv("NLP_ES8_NT")) g->es8_nt = atoi(en) == ES8_NT ? ES8_NT : ES8_NTW;
  if (const char* er = getenv("NLP_ES_RUNS")) g->es_runs = std::min(2, std::max(0, atoi(er)));
  if (const char* rs = getenv("NLP_ES_RS")) g->es_rs = (uint32_t)std::min<long>(ER_RSMAX, std::max(1l, atol(rs)));
  if (const char* lc = getenv("NLP_ES_LCAP")) g->es_lcap = (uint32_t)std::min<long>(EL_CAPMAX, std::max(2l, atol(lc)));
  if (const char* ux = getenv("NLP_HASH_UX")) g->hp_uxf = strcmp(ux, "off") == 0 ? HP_UX_OFF : (uint32_t)atoi(ux);
  if (const char* hd = getenv("NLP_HH_DIRECT")) g->hh_dw = (uint32_t)std::max<long>(0, std::min<long>(HH_DW, atol(hd)));
  if (const char* ha = getenv("NLP_HASH_AA")) g->hp_aa = ha[0] != '0';
  if (const char* hc = getenv("NLP_HASH_HUB_SCAP"))
    g->hh_scap = (uint32_t)std::max<long>(16, std::min<long>(HH_SCAP, atol(hc)));
  if (const char* bf = getenv("NLP_BUCKET_FUSED")) g->split_bucket = bf[0] != '1';
  if (const char* mp = getenv("NLP_MSD_PASSES")) g->msd_force = std::min(2, std::max(0, atoi(mp)));
  if (const char* gr = getenv("NLP_GROUPING")) {
    g->sort_grouping = strcmp(gr, "bucket") != 0;
    g->sort_lsd = strcmp(gr, "lsd") == 0;
  }
  {
    hipDeviceProp_t prop;
    TRY(hipGetDeviceProperties(&prop, g->device));
    const unsigned cus = (unsigned)std::max(prop.multiProcessorCount, 1);
    // grid caps of the ticketed single-pass kernels: at most one resident
    // round of workgroups (the tiles are claimed in order, so correctness does
    // not depend on residency; surplus workgroups would only draw tickets)
    auto occ = [&](const void* k, unsigned* out, int block = NT) -> hipError_t {
      int nb = 0;
      hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, block, 0);
      if (e == hipSuccess) *out = cus * (unsigned)std::max(nb, 1);
      return e;
    };
    TRY(occ((const void*)k_sp_survivors, &g->occ_surv));
    TRY(occ((const void*)k_sp_expand<true>, &g->occ_exp));
    TRY(occ((const void*)k_sp_pass<uint64_t, OS2_IPT>, &g->occ_p64, OS_NT));
    TRY(occ((const void*)k_es_pass<false>, &g->occ_es, ES_NT));
    TRY(occ((const void*)k_es_pass8<false>, &g->occ_es8, ES8_NT));
    TRY(occ((const void*)k_es_pass8<false, ES8_NTW>, &g->occ_es8w, ES8_NTW));
    TRY(occ((const void*)k_hp_batch<false, 1024, 128, true>, &g->occ_hb));
    TRY(occ((const void*)k_sp_pass<uint32_t, OS2_IPT>, &g->occ_p32, OS_NT));
    TRY(occ((const void*)k_sp_pass<uint32_t, OS2_IPT, false, false, GAP_NONE, 11>, &g->occ_p11, OS_NT));
    unsigned a = 0, b = 0;
    TRY(occ((const void*)k_sp_scan<F_Runs<true>, RN_IPT>, &a));
    TRY(occ((const void*)k_sp_scan<F_Runs<false>, RN_IPT>, &b));
    g->occ_run = std::min(a, b);
  }
  g->ws.release();  // drop build scratch; predict grows its own
  TRY(clk.mark("tables_and_setup"));
  return NLP_OK;
}

nlp_status new_graph(int device, nlp_graph** out) {
  nlp_status s = check_device(device);
  if (s != NLP_OK) return s;
  nlp_graph* g = new (std::nothrow) nlp_graph();
  if (!g) return NLP_ERR_NOMEM;
  g->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(&g->host_small, 64 * 8) != hipSuccess ||
      hipHostMalloc(&g->host_ctr, HC_WORDS * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&g->host_ctr_dev, g->host_ctr, 0) != hipSuccess ||
      hipMalloc(&g->d_sticky, 8) != hipSuccess || hipMemset(g->d_sticky, 0, 8) != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  for (int i = 0; i < 8; ++i)
    if (hipEventCreate(&g->ev[i]) != hipSuccess) { destroy_graph(g); return NLP_ERR_DEVICE; }
  // timing-only events skip the system-scope fence (cache writeback) of a
  // default event record; gev[2] ends the call and keeps it (the host reads
  // the counters after it)
  for (int i = 0; i < 5; ++i)
    if (hipEventCreateWithFlags(&g->gev[i], i == 2 ? hipEventDefault : hipEventDisableSystemFence) != hipSuccess) {
      destroy_graph(g);
      return NLP_ERR_DEVICE;
    }
  if (hipEventCreateWithFlags(&g->gev_end, hipEventDisableTiming) != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  *out = g;
  return NLP_OK;
}

// ---------------------------------------------------------------- predict pipeline

struct Params {
  int metric;
  uint32_t H;
  float min_score;
  uint64_t max_edges;
  uint64_t ua, ub;
  uint32_t maxf2 = 0;  // MAXFACTOR2 (predict.hxx:221,295), 0 = off
};

struct Cands {
  uint64_t n = 0;     // candidates currently held in B_CKEY..B_CS
  uint64_t nan = 0;
  uint64_t total = 0; // candidates produced (before pruning)
  uint64_t wedges = 0;
  uint64_t pad = 0;        // path 4: padding entries among the n held (emission window tails, hashpath.hpp hp_flush)
  double hot_ms = 0;       // path 4: device time of the k_hp_batch launches (HIP events around each)
  uint64_t hot_bytes = 0;  // and their algorithmic bytes (counted by the kernel, HPC_HOTB)
  uint32_t hot_launches = 0;
  uint64_t call_bytes = 0; // DESIGN.md §5 model of the bytes of all the call's kernels (path 4)
  // path 4, final prune folded into the order: the n held are unpruned, the
  // order keeps the keys >= kmin and writes the first `keep` (0: pruned)
  uint64_t keep = 0, cap = 0;
  uint32_t kmin = 0;
  uint32_t route = 0;  // path 4: how the final order ran (nlp_timing.order_route)
  int metric = -1;     // the call's (the final order's two-level form is chosen by it)
};

// Group the W wedges of one generator pass, score them and append the
// surviving candidates to the candidate buffer.
__global__ void k_set_u64(uint64_t* p, uint64_t v) { *p = v; }

// Stable LSD sort of (u64 key, u32 value) pairs (values may be null) by the
// 8-bit digits at `shifts` (multiples of 8, least significant first): the
// hist / scan / scatter passes of prims.hpp (a onesweep variant measured
// slower here and was removed in round 4).
nlp_status sort_pairs_os(nlp_graph* g, uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint64_t n,
                         const int* shifts, int np, int* which, hipStream_t st) {
  *which = 0;
  if (n <= 1 || np == 0) return NLP_OK;
  Workspace& ws = g->ws;
  uint64_t *hoff, *scan;
  uint32_t* hist;
  const uint64_t nb = rs_blocks(n);
  TRY(wsget(ws, B_HIST, RS_BINS * nb, &hist));
  TRY(wsget(ws, B_HOFF, RS_BINS * nb, &hoff));
  TRY(wsget(ws, B_SCAN2, scan_scratch_words(std::max<uint64_t>(n, RS_BINS * nb)) + 16, &scan));
  SortScratch sc{hist, hoff, scan, nb};
  TRY(sort_pairs_u64(k0, v0, k1, v1, n, shifts, np, sc, which, st));
  return NLP_OK;
}

// Records: key (u - ubase) << wb | w with u - ubase < 2^ubits (k_wedges), value deg v (AA / RA).
nlp_status group_and_score(nlp_graph* g, const Params& p, uint64_t W, uint64_t* wk, uint32_t* wv, Cands& C,
                           hipStream_t st, uint32_t ubase, int ubits, int wb) {
  Workspace& ws = g->ws;
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  if (W == 0) return NLP_OK;
  uint64_t *wk1, *scan, *rid, *rstart, *rpos, *cnt;
  uint32_t *wv1 = nullptr, *rflag, *rkey, *ru, *rw, *rfl;
  float* rs;
  TRY(wsget(ws, B_WKEY1, W, &wk1));
  if (custom) TRY(wsget(ws, B_WVAL1, W, &wv1));
  TRY(wsget(ws, B_CNT, 8, &cnt));
  // 1. stable sort by (u, w): the bytes of the packed key
  int shifts[8], np = 0;
  for (int b = 0; b < ubits + wb && np < 8; b += 8) shifts[np++] = b;
  int which = 0;
  { nlp_status so = sort_pairs_os(g, wk, custom ? wv : nullptr, wk1, custom ? wv1 : nullptr, W, shifts, np, &which, st);
    if (so != NLP_OK) return so; }
  uint64_t* sk = which ? wk1 : wk;
  uint32_t* sv = which ? wv1 : wv;
  TRY(wsget(ws, B_SCAN2, scan_scratch_words(W) + 16, &scan));  // after the sort (its fallback regrows B_SCAN2)
  // 2. runs of equal (u, w)
  TRY(wsget(ws, B_RFLAG, W, &rflag));
  TRY(wsget(ws, B_RID, W, &rid));
  LAUNCH(k_run_flags, W, st, sk, W, rflag);
  TRY(hipGetLastError());
  TRY(scan_excl_u64<uint32_t>(rflag, W, rid, cnt, scan, st));
  TRY(read_small(g, cnt, 1, st));
  const uint64_t R = g->host_small[0];
  TRY(wsget(ws, B_RSTART, R + 1, &rstart));
  LAUNCH(k_run_starts, W, st, rflag, rid, W, rstart, cnt);
  TRY(hipGetLastError());
  // 3. score every run
  TRY(wsget(ws, B_RKEY, R, &rkey));
  TRY(wsget(ws, B_RU, R, &ru));
  TRY(wsget(ws, B_RW, R, &rw));
  TRY(wsget(ws, B_RS, R, &rs));
  TRY(wsget(ws, B_RFL, R, &rfl));
  TRY(wsget(ws, B_RPOS, R, &rpos));
  const double* ctab = p.metric == M_AA ? g->ctab_aa : g->ctab_ra;
  if (custom)
    LAUNCH(k_score<true>, R, st, rstart, cnt, sk, sv, g->off, g->keys, g->deg, ctab, p.metric, p.min_score, rkey, ru, rw,
           rs, rfl, p.maxf2, g->etab, g->etbits, ubase, wb);
  else
    LAUNCH(k_score<false>, R, st, rstart, cnt, sk, sv, g->off, g->keys, g->deg, ctab, p.metric, p.min_score, rkey, ru,
           rw, rs, rfl, p.maxf2, g->etab, g->etbits, ubase, wb);
  TRY(hipGetLastError());
  // 4. append flagged candidates
  TRY(scan_excl_u64<uint32_t>(rfl, R, rpos, cnt + 1, scan, st));
  TRY(read_small(g, cnt + 1, 1, st));
  const uint64_t add = g->host_small[0];
  uint32_t *ckey, *cu, *cw;
  float* cs;
  uint64_t need = C.n + add;
  // grow the candidate buffer preserving contents
  if (need * 4 > ws.bytes[B_CKEY]) {
    uint32_t *ok = (uint32_t*)ws.p[B_CKEY], *ou = (uint32_t*)ws.p[B_CU], *ow = (uint32_t*)ws.p[B_CW];
    float* os = (float*)ws.p[B_CS];
    uint64_t cap = std::max<uint64_t>(need, 2 * C.n);
    uint32_t *nk, *nu, *nw;
    float* ns;
    TRY(wsget(ws, B_TKEY, cap, &nk));
    TRY(wsget(ws, B_TU, cap, &nu));
    TRY(wsget(ws, B_TW, cap, &nw));
    TRY(wsget(ws, B_TS, cap, &ns));
    if (C.n) {
      TRY(hipMemcpyAsync(nk, ok, C.n * 4, hipMemcpyDeviceToDevice, st));
      TRY(hipMemcpyAsync(nu, ou, C.n * 4, hipMemcpyDeviceToDevice, st));
      TRY(hipMemcpyAsync(nw, ow, C.n * 4, hipMemcpyDeviceToDevice, st));
      TRY(hipMemcpyAsync(ns, os, C.n * 4, hipMemcpyDeviceToDevice, st));
    }
    std::swap(ws.p[B_CKEY], ws.p[B_TKEY]); std::swap(ws.bytes[B_CKEY], ws.bytes[B_TKEY]);
    std::swap(ws.p[B_CU], ws.p[B_TU]); std::swap(ws.bytes[B_CU], ws.bytes[B_TU]);
    std::swap(ws.p[B_CW], ws.p[B_TW]); std::swap(ws.bytes[B_CW], ws.bytes[B_TW]);
    std::swap(ws.p[B_CS], ws.p[B_TS]); std::swap(ws.bytes[B_CS], ws.bytes[B_TS]);
  }
  TRY(wsget(ws, B_CKEY, need, &ckey));
  TRY(wsget(ws, B_CU, need, &cu));
  TRY(wsget(ws, B_CW, need, &cw));
  TRY(wsget(ws, B_CS, need, &cs));
  LAUNCH(k_compact_cands, R, st, rfl, rpos, cnt, rkey, ru, rw, rs, C.n, ckey, cu, cw, cs);
  TRY(hipGetLastError());
  C.n += add;
  C.total += add;
  return NLP_OK;
}

// Radix-select the canonical top `k` of the candidate buffer (in place).  The
// buffer is in (u, w) order, so "first `quota` ties in buffer order" is the
// canonical (u asc, w asc) tie fill.
nlp_status prune_to(nlp_graph* g, Cands& C, uint64_t k, hipStream_t st) {
  if (C.n <= k) return NLP_OK;
  Workspace& ws = g->ws;
  uint32_t *ckey = (uint32_t*)ws.p[B_CKEY], *cu = (uint32_t*)ws.p[B_CU], *cw = (uint32_t*)ws.p[B_CW];
  float* cs = (float*)ws.p[B_CS];
  uint32_t *selhist, *tie, *keep;
  uint64_t *sel, *trank, *kpos, *scan, *cnt;
  TRY(wsget(ws, B_SELHIST, SEL_BINS, &selhist));
  TRY(wsget(ws, B_SEL, 8, &sel));
  TRY(wsget(ws, B_TIE, C.n, &tie));
  TRY(wsget(ws, B_TRANK, C.n, &trank));
  TRY(wsget(ws, B_KEEP, C.n, &keep));
  TRY(wsget(ws, B_KPOS, C.n, &kpos));
  TRY(wsget(ws, B_SCAN2, scan_scratch_words(C.n) + 16, &scan));
  TRY(wsget(ws, B_CNT, 8, &cnt));
  // candidate count lives on the device for the select kernels
  g->host_small[8] = C.n;
  g->host_small[9] = 0;  // sel[0] prefix
  g->host_small[10] = k; // sel[1] rank
  g->host_small[11] = 0; // sel[2] above
  g->host_small[12] = 0;
  TRY(hipMemcpyAsync(cnt + 4, &g->host_small[8], 8, hipMemcpyHostToDevice, st));
  TRY(hipMemcpyAsync(sel, &g->host_small[9], 32, hipMemcpyHostToDevice, st));
  TRY(hipMemsetAsync(selhist, 0, SEL_BINS * 4, st));
  for (int pass = 0; pass < 3; ++pass) {
    LAUNCH(k_sel_hist, C.n, st, ckey, cnt + 4, pass, sel, selhist);
    hipLaunchKernelGGL(k_sel_pick, dim3(1), dim3(NT), 0, st, selhist, pass, sel);
    TRY(hipGetLastError());
  }
  LAUNCH(k_tie_flags, C.n, st, ckey, C.n, sel, tie);
  TRY(hipGetLastError());
  TRY(scan_excl_u64<uint32_t>(tie, C.n, trank, nullptr, scan, st));
  LAUNCH(k_keep_flags, C.n, st, ckey, C.n, sel, trank, keep);
  TRY(hipGetLastError());
  TRY(scan_excl_u64<uint32_t>(keep, C.n, kpos, cnt + 5, scan, st));
  uint32_t *nk, *nu, *nw;
  float* ns;
  TRY(wsget(ws, B_TKEY, k, &nk));
  TRY(wsget(ws, B_TU, k, &nu));
  TRY(wsget(ws, B_TW, k, &nw));
  TRY(wsget(ws, B_TS, k, &ns));
  LAUNCH(k_compact_cands, C.n, st, keep, kpos, cnt + 4, ckey, cu, cw, cs, (uint64_t)0, nk, nu, nw, ns);
  TRY(hipGetLastError());
  std::swap(ws.p[B_CKEY], ws.p[B_TKEY]); std::swap(ws.bytes[B_CKEY], ws.bytes[B_TKEY]);
  std::swap(ws.p[B_CU], ws.p[B_TU]); std::swap(ws.bytes[B_CU], ws.bytes[B_TU]);
  std::swap(ws.p[B_CW], ws.p[B_TW]); std::swap(ws.bytes[B_CW], ws.bytes[B_TW]);
  std::swap(ws.p[B_CS], ws.p[B_TS]); std::swap(ws.bytes[B_CS], ws.bytes[B_TS]);
  C.n = k;
  return NLP_OK;
}

// Stable sort of the candidate buffer by score key descending -> edges.
nlp_status order_into(nlp_graph* g, Cands& C, EdgeOut* d_out, hipStream_t st) {
  if (C.n == 0) return NLP_OK;
  Workspace& ws = g->ws;
  uint64_t *k0, *k1;
  uint32_t *v0, *v1;
  TRY(wsget(ws, B_SK0, C.n, &k0));
  TRY(wsget(ws, B_SK1, C.n, &k1));
  TRY(wsget(ws, B_SV0, C.n, &v0));
  TRY(wsget(ws, B_SV1, C.n, &v1));
  LAUNCH(k_desc_keys, C.n, st, (const uint32_t*)ws.p[B_CKEY], C.n, k0, v0);
  TRY(hipGetLastError());
  int shifts[4] = {0, 8, 16, 24};
  int which = 0;
  { nlp_status so = sort_pairs_os(g, k0, v0, k1, v1, C.n, shifts, 4, &which, st); if (so != NLP_OK) return so; }
  LAUNCH(k_gather_edges, C.n, st, which ? v1 : v0, C.n, (const uint32_t*)ws.p[B_CU], (const uint32_t*)ws.p[B_CW],
         (const float*)ws.p[B_CS], d_out);
  TRY(hipGetLastError());
  return NLP_OK;
}

nlp_status count_nan(nlp_graph* g, Cands& C, hipStream_t st) {
  uint64_t* cnt;
  TRY(wsget(g->ws, B_CNT, 8, &cnt));
  TRY(hipMemsetAsync(cnt + 6, 0, 8, st));
  if (C.n) LAUNCH(k_count_key0, C.n, st, (const uint32_t*)g->ws.p[B_CKEY], C.n, (unsigned long long*)(cnt + 6));
  TRY(hipGetLastError());
  TRY(read_small(g, cnt + 6, 1, st));
  C.nan = g->host_small[0];
  return NLP_OK;
}


// ================================================================ v1 pipeline
// Arena layout (u64 words): [0,16) counters, [16,32) tickets (u32 pairs),
// then look-back descriptors of the scans, each region tiles(n) words.
struct Arena {
  uint64_t* base = nullptr;
  uint64_t words = 0;
  uint64_t* ctr() const { return base; }
  uint32_t* ticket(int i) const { return (uint32_t*)(base + 16) + i; }
};

inline uint64_t tiles_of(uint64_t n) { return (n + LB_TILE - 1) / LB_TILE + 1; }

// zero the arena and set the initial counters (one kernel)
nlp_status arena_init(nlp_graph* g, int id, uint64_t desc_words, Arena& A, const uint64_t* init, hipStream_t st) {
  A.words = 32 + desc_words;
  TRY(wsget(g->ws, id, A.words, &A.base));
  CtrInit ci;
  for (int i = 0; i < NCTR; ++i) ci.v[i] = init ? init[i] : 0;
  hipLaunchKernelGGL(k_arena_init, dim3(std::min<uint64_t>(1024, (A.words + NT - 1) / NT)), dim3(NT), 0, st, A.base,
                     A.words, ci);
  TRY(hipGetLastError());
  return NLP_OK;
}

GraphView view_of(nlp_graph* g, int metric, uint32_t maxf2 = 0) {
  return GraphView{g->off,  g->keys, g->deg, g->toff, g->tkeys, metric == M_AA ? g->ctab_aa : g->ctab_ra,
                   g->efilt, g->efbits, maxf2, g->etab, g->etbits};
}

template <class F>
hipError_t launch_scan(const F& f, const uint64_t* d_n, uint64_t n_upper, uint32_t* ticket, uint64_t* desc,
                       uint32_t* err, uint64_t* total, hipStream_t st) {
  LbState ls{ticket, desc, err};
  hipLaunchKernelGGL(k_lb_scan<F>, dim3(lb_grid(n_upper)), dim3(NT), 0, st, f, d_n, ls, total);
  return hipGetLastError();
}

struct StageBufs {
  Stage st;
  uint64_t* bucket;
  uint32_t* big;
};

nlp_status stage_bufs(nlp_graph* g, uint64_t capW, uint64_t nbig, StageBufs& b) {
  Workspace& ws = g->ws;
  TRY(wsget(ws, B_BUCKET, capW, &b.bucket));
  TRY(wsget(ws, B_SKEY, capW, &b.st.key));
  TRY(wsget(ws, B_SU, capW, &b.st.u));
  TRY(wsget(ws, B_SW, capW, &b.st.w));
  TRY(wsget(ws, B_SS, capW, &b.st.s));
  TRY(wsget(ws, B_SFLAG, capW, &b.st.flag));
  TRY(wsget(ws, B_BIG, nbig, &b.big));
  return NLP_OK;
}

// Make sure the candidate buffer holds `need` entries, preserving `keep`.
nlp_status cand_reserve(nlp_graph* g, uint64_t need, uint64_t keep, hipStream_t st) {
  Workspace& ws = g->ws;
  if (need * 4 <= ws.bytes[B_CKEY] && need * 4 <= ws.bytes[B_CU] && need * 4 <= ws.bytes[B_CW] &&
      need * 4 <= ws.bytes[B_CS])
    return NLP_OK;
  uint32_t *nk, *nu, *nw;
  float* ns;
  uint64_t cap = std::max<uint64_t>(need, 2 * keep);
  TRY(wsget(ws, B_TKEY, cap, &nk));
  TRY(wsget(ws, B_TU, cap, &nu));
  TRY(wsget(ws, B_TW, cap, &nw));
  TRY(wsget(ws, B_TS, cap, &ns));
  if (keep) {
    TRY(hipMemcpyAsync(nk, ws.p[B_CKEY], keep * 4, hipMemcpyDeviceToDevice, st));
    TRY(hipMemcpyAsync(nu, ws.p[B_CU], keep * 4, hipMemcpyDeviceToDevice, st));
    TRY(hipMemcpyAsync(nw, ws.p[B_CW], keep * 4, hipMemcpyDeviceToDevice, st));
    TRY(hipMemcpyAsync(ns, ws.p[B_CS], keep * 4, hipMemcpyDeviceToDevice, st));
  }
  std::swap(ws.p[B_CKEY], ws.p[B_TKEY]); std::swap(ws.bytes[B_CKEY], ws.bytes[B_TKEY]);
  std::swap(ws.p[B_CU], ws.p[B_TU]); std::swap(ws.bytes[B_CU], ws.bytes[B_TU]);
  std::swap(ws.p[B_CW], ws.p[B_TW]); std::swap(ws.bytes[B_CW], ws.bytes[B_TW]);
  std::swap(ws.p[B_CS], ws.p[B_TS]); std::swap(ws.bytes[B_CS], ws.bytes[B_TS]);
  return NLP_OK;
}

// Path 1 (intermediate-centric) with per-source buckets.  F_OVERFLOW is
// handled here by growing and re-running; F_TOOBIG is returned to the caller,
// which then uses the radix path.  ucnt/cursor are kept all-zero between calls.
nlp_status run_path1_v1(nlp_graph* g, const Params& p, Cands& C, uint64_t* flags_out, bool* over_budget,
                        hipStream_t st) {
  const uint64_t S = g->span;
  const uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S), nU = ub - ua;
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  const GraphView gv = view_of(g, p.metric, p.maxf2);
  Workspace& ws = g->ws;
  *over_budget = false;
  // zero-invariant counters: allocate (and zero) once
  if (ws.bytes[B_UCNT] < S * 4 || ws.bytes[B_IEP] < S * 4) {
    uint32_t *a, *b;
    TRY(wsget(ws, B_UCNT, S, &a));
    TRY(wsget(ws, B_IEP, S, &b));
    TRY(hipMemsetAsync(a, 0, S * 4, st));
    TRY(hipMemsetAsync(b, 0, S * 4, st));
  }
  uint32_t* ucnt = (uint32_t*)ws.p[B_UCNT];
  uint32_t* cursor = (uint32_t*)ws.p[B_IEP];
  for (int attempt = 0; attempt < 3; ++attempt) {
    const uint64_t capW = g->capW;
    uint64_t* uoff;
    TRY(wsget(ws, B_UOFF, S, &uoff));
    StageBufs sb;
    nlp_status s = stage_bufs(g, capW, 0, sb);
    if (s != NLP_OK) return s;
    BigItem* big;
    TRY(wsget(ws, B_BIG, std::max<uint64_t>(nU, 1), &big));
    s = cand_reserve(g, capW, 0, st);
    if (s != NLP_OK) return s;
    uint32_t *ck = (uint32_t*)ws.p[B_CKEY], *cu = (uint32_t*)ws.p[B_CU], *cw = (uint32_t*)ws.p[B_CW];
    float* cs = (float*)ws.p[B_CS];
    constexpr int IPT_S = 16, IPT_W = 4;
    const uint64_t aU = (nU + NT * IPT_S - 1) / (NT * IPT_S) + 1, aW = (capW + NT * IPT_W - 1) / (NT * IPT_W) + 1;
    Arena A;
    uint64_t init[NCTR] = {};
    init[C_N_URANGE] = nU;
    init[10] = S;
    s = arena_init(g, B_ARENA, 0, A, init, st);
    if (s != NLP_OK) return s;
    uint64_t* ctr = A.ctr();
    uint64_t* aggs;
    TRY(wsget(ws, B_ARENA2, aU + aW, &aggs));
    uint64_t* gU = aggs;
    uint64_t* gW = gU + aU;
    hipLaunchKernelGGL(k_p1_pass<false>, dim3(p1_grid(S)), dim3(NT), 0, st, gv, S, p.H, ua, ub, ucnt, (const uint64_t*)nullptr, capW, sb.bucket, ctr);
    TRY(hipGetLastError());
    TRY((rts_scan<F_UOff, IPT_S>(F_UOff{ucnt, uoff, ua}, &ctr[C_N_URANGE], nU, gU, &ctr[C_W], st)));
    hipLaunchKernelGGL(k_p1_pass<true>, dim3(p1_grid(S)), dim3(NT), 0, st, gv, S, p.H, ua, ub, cursor, (const uint64_t*)uoff, capW, sb.bucket, ctr);
    TRY(hipGetLastError());
    BucketsP1 bk{uoff, ucnt};
    const unsigned gtiles = (unsigned)std::min<uint64_t>(std::max<uint64_t>((nU + GT_TILE - 1) / GT_TILE, 1), 65535);
    if (custom) {
      hipLaunchKernelGGL((k_group_tiles<BucketsP1, true>), dim3(gtiles), dim3(NT), 0, st, gv, bk, ua, ub, p.metric,
                         p.min_score, sb.bucket, capW, sb.st, big, ctr, ucnt, cursor);
      hipLaunchKernelGGL((k_group_big<true>), dim3(256), dim3(NT), 0, st, gv, p.metric, p.min_score, sb.bucket, sb.st,
                         (const BigItem*)big, ctr);
      LAUNCH_FULL(k_score_runs<true>, capW, st, gv, p.metric, p.min_score, ctr, capW, sb.st);
    } else {
      hipLaunchKernelGGL((k_group_tiles<BucketsP1, false>), dim3(gtiles), dim3(NT), 0, st, gv, bk, ua, ub, p.metric,
                         p.min_score, sb.bucket, capW, sb.st, big, ctr, ucnt, cursor);
      hipLaunchKernelGGL((k_group_big<false>), dim3(256), dim3(NT), 0, st, gv, p.metric, p.min_score, sb.bucket, sb.st,
                         (const BigItem*)big, ctr);
      LAUNCH_FULL(k_score_runs<false>, capW, st, gv, p.metric, p.min_score, ctr, capW, sb.st);
    }
    TRY(hipGetLastError());
    hipLaunchKernelGGL(k_clamp_n, dim3(1), dim3(64), 0, st, ctr, (uint64_t)C_W, capW, (uint64_t)11);
    TRY((rts_scan<F_Compact, IPT_W>(F_Compact{sb.st, ck, cu, cw, cs, ctr, &ctr[C_NAN]}, &ctr[11], capW, gW,
                                    &ctr[C_C], st)));
    TRY(hipMemcpyAsync(g->host_small, ctr, NCTR * 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    const uint64_t* h = g->host_small;
    if (h[C_FLAGS] & F_OVERFLOW) {
      // the grouping did not run: counters are dirty
      TRY(hipMemsetAsync(ucnt, 0, S * 4, st));
      TRY(hipMemsetAsync(cursor, 0, S * 4, st));
      uint64_t W = h[C_W];
      if (W > g->wedge_budget) { *over_budget = true; return NLP_OK; }
      if (W > g->capW) g->capW = W + W / 4 + 1024;
      continue;
    }
    if (h[C_W] > g->wedge_budget) { *over_budget = true; return NLP_OK; }
    *flags_out = h[C_FLAGS];
    C.n = h[C_C];
    C.total = h[C_C];
    C.nan = h[C_NAN];
    C.wedges += h[C_W];
    return NLP_OK;
  }
  return NLP_ERR_DEVICE;
}

// Stable descending order of the candidate buffer by score key -> edges (onesweep).
nlp_status order_v1(nlp_graph* g, Cands& C, EdgeOut* d_out, hipStream_t st) {
  if (C.n == 0) return NLP_OK;
  Workspace& ws = g->ws;
  uint32_t *k0, *k1, *v0, *v1;
  TRY(wsget(ws, B_OK0, C.n, &k0));
  TRY(wsget(ws, B_OK1, C.n, &k1));
  TRY(wsget(ws, B_OV0, C.n, &v0));
  TRY(wsget(ws, B_OV1, C.n, &v1));
  const uint64_t nt = (C.n + OS_TILE - 1) / OS_TILE;
  Arena A;
  uint64_t init[NCTR] = {};
  init[0] = C.n;
  nlp_status s = arena_init(g, B_ARENA2, 512 + 4 * nt * RS_BINS, A, init, st);
  if (s != NLP_OK) return s;
  uint64_t* ctr = A.ctr();
  uint32_t* ghist = (uint32_t*)(A.base + 32);  // 4 x 256 u32 = 512 words... (uses 512 u64 of space)
  uint64_t* desc = A.base + 32 + 512;
  uint32_t* err = (uint32_t*)&ctr[1];
  LAUNCH(k_desc_keys32, C.n, st, (const uint32_t*)ws.p[B_CKEY], C.n, k0, v0);
  TRY(hipGetLastError());
  // 4 workgroups per CU: the score keys' high digits are few (ties), and 64
  // workgroups serialised on their LDS atomics (C4 JAC H=16: 4.8 ms for 1.9e8 keys)
  hipLaunchKernelGGL(k_os_hist, dim3(std::min<uint64_t>(1024, grid_for(C.n))), dim3(NT), 0, st, k0, ctr, ghist);
  TRY(hipGetLastError());
  uint32_t *ka = k0, *va = v0, *kb = k1, *vb = v1;
  for (int pass = 0; pass < 4; ++pass) {
    hipLaunchKernelGGL(k_os_pass, dim3((unsigned)nt), dim3(NT), 0, st, ka, va, kb, vb, ctr, 8 * pass,
                       ghist + pass * RS_BINS, A.ticket(pass), desc + (uint64_t)pass * nt * RS_BINS, err);
    TRY(hipGetLastError());
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  LAUNCH(k_gather_edges, C.n, st, va, C.n, (const uint32_t*)ws.p[B_CU], (const uint32_t*)ws.p[B_CW],
         (const float*)ws.p[B_CS], d_out);
  TRY(hipGetLastError());
  return NLP_OK;
}

// Path 1 generator: returns NLP_ERR_CAPACITY through *fits = false when the
// wedge count exceeds the budget (then path 2 runs instead).
nlp_status run_path1(nlp_graph* g, const Params& p, Cands& C, bool* fits, hipStream_t st) {
  Workspace& ws = g->ws;
  const uint64_t S = g->span;
  uint32_t *c32, *ev, *eu, *ewc, *efirst, *wv = nullptr;
  uint64_t *ioff, *woff, *scan, *cnt, *wk;
  TRY(wsget(ws, B_C32, S, &c32));
  TRY(wsget(ws, B_IOFF, S, &ioff));
  TRY(wsget(ws, B_SCAN, scan_scratch_words(S) + 16, &scan));
  TRY(wsget(ws, B_CNT, 8, &cnt));
  LAUNCH(k_p1_vcount, S, st, g->deg, g->toff, S, p.H, c32);
  TRY(hipGetLastError());
  TRY(scan_excl_u64<uint32_t>(c32, S, ioff, cnt, scan, st));
  TRY(read_small(g, cnt, 1, st));
  const uint64_t E = g->host_small[0];
  *fits = true;
  if (E == 0) return NLP_OK;
  TRY(wsget(ws, B_EV, E, &ev));
  TRY(wsget(ws, B_EU, E, &eu));
  TRY(wsget(ws, B_EWC, E, &ewc));
  TRY(wsget(ws, B_EFIRST, E, &efirst));
  TRY(wsget(ws, B_WOFF, E, &woff));
  LAUNCH(k_p1_inedges, E, st, ioff, S, cnt, g->toff, g->tkeys, g->off, g->keys, g->deg, p.ua, p.ub, ev, eu, ewc, efirst);
  TRY(hipGetLastError());
  TRY(wsget(ws, B_SCAN, scan_scratch_words(std::max(S, E)) + 16, &scan));
  TRY(scan_excl_u64<uint32_t>(ewc, E, woff, cnt + 1, scan, st));
  TRY(read_small(g, cnt + 1, 1, st));
  const uint64_t W = g->host_small[0];
  if (W > g->wedge_budget) { *fits = false; return NLP_OK; }
  C.wedges += W;
  if (W == 0) return NLP_OK;
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  TRY(wsget(ws, B_WKEY0, W, &wk));
  if (custom) TRY(wsget(ws, B_WVAL0, W, &wv));
  const uint64_t ua1 = std::min(p.ua, S), ub1 = std::min(p.ub, S);
  const int wb1 = bits_for(S - 1), ubits1 = bits_for(ub1 > ua1 ? ub1 - ua1 - 1 : 0);
  if (custom)
    hipLaunchKernelGGL(k_wedges<true>, dim3((unsigned)std::min<uint64_t>((W + WG_TILE - 1) / WG_TILE, 65535)), dim3(NT), 0, st, woff, E, cnt + 1, (uint64_t)0, ev, eu, efirst, g->off, g->keys, g->deg, wk, wv,
           (uint32_t)ua1, wb1);
  else
    hipLaunchKernelGGL(k_wedges<false>, dim3((unsigned)std::min<uint64_t>((W + WG_TILE - 1) / WG_TILE, 65535)), dim3(NT), 0, st, woff, E, cnt + 1, (uint64_t)0, ev, eu, efirst, g->off, g->keys, g->deg, wk, wv,
           (uint32_t)ua1, wb1);
  TRY(hipGetLastError());
  return group_and_score(g, p, W, wk, wv, C, st, (uint32_t)ua1, ubits1, wb1);
}

// Path 2 generator: source range [ua, ub) in chunks of <= wedge_budget wedges
// (a single source vertex larger than the budget forms its own chunk).
nlp_status run_path2(nlp_graph* g, const Params& p, Cands& C, uint32_t* nchunks, hipStream_t st) {
  Workspace& ws = g->ws;
  const uint64_t S = g->span;
  uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S);
  uint64_t hb[2];
  TRY(hipMemcpyAsync(&g->host_small[16], g->off + ua, 8, hipMemcpyDeviceToHost, st));
  TRY(hipMemcpyAsync(&g->host_small[17], g->off + ub, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  hb[0] = g->host_small[16];
  hb[1] = g->host_small[17];
  const uint64_t e0 = hb[0], e1 = hb[1];
  const uint64_t E = e1 - e0;
  *nchunks = 0;
  if (E == 0) return NLP_OK;
  uint32_t *ev, *eu, *ewc, *efirst, *wv = nullptr;
  uint64_t *woff, *scan, *cnt, *wk;
  TRY(wsget(ws, B_EV, E, &ev));
  TRY(wsget(ws, B_EU, E, &eu));
  TRY(wsget(ws, B_EWC, E, &ewc));
  TRY(wsget(ws, B_EFIRST, E, &efirst));
  TRY(wsget(ws, B_WOFF, E + 1, &woff));
  TRY(wsget(ws, B_SCAN, scan_scratch_words(E + 1) + 16, &scan));
  TRY(wsget(ws, B_CNT, 8, &cnt));
  LAUNCH(k_p2_edges, E, st, g->off, g->keys, g->deg, S, e0, e1, p.H, ev, eu, ewc, efirst, (const uint32_t*)g->tile_row,
         (uint64_t)HP_WTILE, g->nnz);
  TRY(hipGetLastError());
  TRY(scan_excl_u64<uint32_t>(ewc, E, woff, cnt + 1, scan, st));
  TRY(hipMemcpyAsync(woff + E, cnt + 1, 8, hipMemcpyDeviceToDevice, st));  // woff[E] = W
  TRY(read_small(g, cnt + 1, 1, st));
  const uint64_t Wall = g->host_small[0];
  C.wedges += Wall;
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  // chunk loop over edge slots [a, b) aligned to source rows
  uint64_t a = 0;
  std::vector<uint64_t> row_starts;
  while (a < E && Wall > 0) {
    uint64_t wa = 0, bnd = E;
    TRY(hipMemcpyAsync(&g->host_small[18], woff + a, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    wa = g->host_small[18];
    if (Wall - wa > g->wedge_budget) {
      // first edge slot whose offset exceeds wa + budget, then back to its row start
      hipLaunchKernelGGL(k_find_chunk_end, dim3(1), dim3(64), 0, st, woff, E + 1, wa + g->wedge_budget, cnt + 2);
      TRY(hipGetLastError());
      TRY(read_small(g, cnt + 2, 1, st));
      uint64_t e = g->host_small[0];  // first slot with woff > target (1..E+1)
      uint64_t slot = e - 1;          // last slot with woff <= target
      if (slot > E) slot = E;
      // row containing edge e0 + slot: find via offsets on the host side copy
      uint64_t eg = e0 + slot;
      // binary search offsets on the device would need another kernel; use a
      // small host bisection over device reads
      uint64_t lo = ua, hi = ub;  // largest u with off[u] <= eg
      while (hi - lo > 1) {
        uint64_t mid = (lo + hi) / 2;
        TRY(hipMemcpy(&g->host_small[19], g->off + mid, 8, hipMemcpyDeviceToHost));
        if (g->host_small[19] <= eg) lo = mid; else hi = mid;
      }
      TRY(hipMemcpy(&g->host_small[19], g->off + lo, 8, hipMemcpyDeviceToHost));
      uint64_t rs = g->host_small[19] - e0;
      if (rs <= a) {  // a single row larger than the budget: take the whole row
        TRY(hipMemcpy(&g->host_small[19], g->off + lo + 1, 8, hipMemcpyDeviceToHost));
        rs = g->host_small[19] - e0;
      }
      bnd = std::min(rs, E);
    }
    TRY(hipMemcpyAsync(&g->host_small[20], woff + bnd, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    const uint64_t wb = g->host_small[20];
    const uint64_t W = wb - wa;
    if (W) {
      TRY(wsget(ws, B_WKEY0, W, &wk));
      if (custom) TRY(wsget(ws, B_WVAL0, W, &wv));
      // cnt[3] = wb for the grid-stride bound
      g->host_small[21] = wb;
      TRY(hipMemcpyAsync(cnt + 3, &g->host_small[21], 8, hipMemcpyHostToDevice, st));
      const int wb2 = bits_for(S - 1), ubits2 = bits_for(ub > ua ? ub - ua - 1 : 0);
      if (custom)
        hipLaunchKernelGGL(k_wedges<true>, dim3((unsigned)std::min<uint64_t>((W + WG_TILE - 1) / WG_TILE, 65535)), dim3(NT), 0, st, woff, E, cnt + 3, wa, ev, eu, efirst, g->off, g->keys, g->deg, wk, wv,
               (uint32_t)ua, wb2);
      else
        hipLaunchKernelGGL(k_wedges<false>, dim3((unsigned)std::min<uint64_t>((W + WG_TILE - 1) / WG_TILE, 65535)), dim3(NT), 0, st, woff, E, cnt + 3, wa, ev, eu, efirst, g->off, g->keys, g->deg, wk, wv,
               (uint32_t)ua, wb2);
      TRY(hipGetLastError());
      nlp_status s = group_and_score(g, p, W, wk, wv, C, st, (uint32_t)ua, ubits2, wb2);
      if (s != NLP_OK) return s;
      if (C.n > 2 * p.max_edges + (1u << 20)) {
        s = prune_to(g, C, p.max_edges, st);
        if (s != NLP_OK) return s;
      }
    }
    ++*nchunks;
    a = bnd;
  }
  return NLP_OK;
}

// ================================================================ path 3 (hash accumulation)
// hashpath.hpp: source rows binned by their wedge bound W(u), accumulated in
// LDS / global hash tables, candidates emitted unordered above the running
// threshold tau and pruned to the canonical top k between chunks of rows.

// Wedge scratch of k_hp_part (bins 2 and 3), allocated once per graph: 2 x
// hp_scap words per workgroup (w and, for AA / RA, v).
nlp_status hp_alloc_scratch(nlp_graph* g) {
  if (g->hp_scratch) return NLP_OK;
  size_t fr = 0, tot = 0;
  TRY(hipMemGetInfo(&fr, &tot));
  g->hp_gp = 256;
  uint64_t scap = g->hp_scap_force ? g->hp_scap_force : (1ull << 22);  // 8 GB when a sixteenth of HBM is free
  while (scap > 4096 && (uint64_t)g->hp_gp * scap * 8 > fr / 16) scap >>= 1;
  g->hp_scap = scap;
  TRY(hipMalloc(&g->hp_scratch, (uint64_t)g->hp_gp * scap * 8));
  return NLP_OK;
}

// Prune the (unordered) candidate buffer to the canonical top k:
// radix-select the k-th key, keep every key above it and the first ties in
// (u, w) order.  Returns the k-th key in *kth.
// fuse (the call's last prune): when the keys at or above the k-th are few
// beyond k (the tie set small) and the 8-byte order may take them, nothing is
// split -- C.keep / C.kmin hand the unpruned buffer to hp_final_order, which
// sorts the keys >= kmin and writes the first k (the canonical tie rule is the
// sort order).
nlp_status hp_prune(nlp_graph* g, Cands& C, uint64_t k, uint64_t cap, uint32_t* kth, hipStream_t st,
                    bool fuse = false) {
  Workspace& ws = g->ws;
  const uint64_t n = C.n;
  uint32_t *ckey = (uint32_t*)ws.p[B_CKEY], *cu = (uint32_t*)ws.p[B_CU], *cw = (uint32_t*)ws.p[B_CW];
  float* cs = (float*)ws.p[B_CS];
  uint32_t* selhist;
  uint64_t *sel, *small;
  TRY(wsget(ws, B_SELHIST, SEL_BINS, &selhist));
  TRY(wsget(ws, B_SEL, 8, &sel));
  TRY(wsget(ws, B_HP_SMALL, 72, &small));  // [64, 68): NLP_TRACE_BATCH phase ticks
  uint64_t* h = g->host_small;
  h[8] = n;
  h[9] = 0;  // sel: prefix, rank, above, key
  h[10] = k;
  h[11] = 0;
  h[12] = 0;
  TRY(hipMemcpyAsync(small + 32, &h[8], 8, hipMemcpyHostToDevice, st));
  TRY(hipMemcpyAsync(sel, &h[9], 32, hipMemcpyHostToDevice, st));
  TRY(hipMemsetAsync(selhist, 0, SEL_BINS * 4, st));
  TRY(hipMemsetAsync(small + 40, 0, 16, st));
  for (int pass = 0; pass < 3; ++pass) {
    LAUNCH(k_sel_hist, n, st, ckey, small + 32, pass, sel, selhist);
    hipLaunchKernelGGL(k_sel_pick, dim3(1), dim3(NT), 0, st, selhist, pass, sel);
    TRY(hipGetLastError());
  }
  if (fuse && g->es_k8 == 1 && n >= ES8_MIN && n < (1ull << 32)) {
    TRY(hipMemcpyAsync(&h[16], sel, 40, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    const uint64_t above = h[18], key = h[19], ties = h[20];
    if (key > 0 && above < k && above + ties >= k && above + ties <= k + std::max<uint64_t>(k / 16, 1ull << 16)) {
      *kth = (uint32_t)key;
      C.keep = k;
      C.kmin = (uint32_t)key;
      C.cap = cap;
      C.call_bytes += 12 * n;  // three select histograms
      return NLP_OK;
    }
  }
  uint32_t *nk, *nu, *nw, *ti0, *ti1;
  float* ns;
  uint64_t *tk0, *tk1;
  // the target becomes the candidate buffer: same capacity
  TRY(wsget(ws, B_TKEY, std::max<uint64_t>(cap, 1), &nk));
  TRY(wsget(ws, B_TU, std::max<uint64_t>(cap, 1), &nu));
  TRY(wsget(ws, B_TW, std::max<uint64_t>(cap, 1), &nw));
  TRY(wsget(ws, B_TS, std::max<uint64_t>(cap, 1), &ns));
  TRY(wsget(ws, B_HP_TIEK0, n, &tk0));
  TRY(wsget(ws, B_HP_TIEI0, n, &ti0));
  hipLaunchKernelGGL(k_hp_split, dim3((unsigned)std::min<uint64_t>(std::max<uint64_t>(n / (NT * HP_SPLIT_IPL), 1), 2048)),
                     dim3(NT), 0, st, ckey, cu, cw, cs, n, sel, nk, nu, nw, ns, tk0, ti0,
                     (unsigned long long*)(small + 40));
  TRY(hipGetLastError());
  TRY(hipMemcpyAsync(&h[16], sel, 32, hipMemcpyDeviceToHost, st));
  TRY(hipMemcpyAsync(&h[20], small + 40, 16, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  const uint64_t quota = h[17], above = h[18], ties = h[21];
  *kth = (uint32_t)h[19];
  if (above != h[20] || quota > ties || above + quota != k) return NLP_ERR_DEVICE;
  const uint32_t* take_idx = ti0;
  const int svb = bits_for(g->span - 1);
  if (ties > quota && quota > 0 && 2 * svb <= 4 * TS_BITS) {
    // the quota smallest ties in (u, w) order by radix select (k_ts_*), in any order
    uint32_t* th;
    uint64_t* tst;
    TRY(wsget(ws, B_TSHIST, TS_BINS, &th));  // zeroed here, then by every k_ts_pick
    TRY(hipMemsetAsync(th, 0, TS_BINS * 4, st));
    tst = small + 48;  // [48] prefix, [49] rank, [50] placed count
    h[24] = 0;
    h[25] = quota;
    h[26] = 0;
    TRY(hipMemcpyAsync(tst, &h[24], 24, hipMemcpyHostToDevice, st));
    const unsigned gh = (unsigned)std::min<uint64_t>(std::max<uint64_t>(ties / (NT * 16), 1), 1024);
    for (int d = 3; d >= 0; --d) {
      hipLaunchKernelGGL(k_ts_hist, dim3(gh), dim3(NT), 0, st, (const uint64_t*)tk0, ties, svb, d * TS_BITS,
                         (const uint64_t*)tst, th);
      hipLaunchKernelGGL(k_ts_pick, dim3(1), dim3(NT), 0, st, th, tst);
      TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(k_ts_take, dim3((unsigned)std::min<uint64_t>(std::max<uint64_t>(ties / (NT * 8), 1), 2048)),
                       dim3(NT), 0, st, (const uint64_t*)tk0, (const uint32_t*)ti0, ties, svb, (const uint64_t*)tst,
                       above, ckey, cu, cw, cs, nk, nu, nw, ns, (unsigned long long*)(tst + 2));
    TRY(hipGetLastError());
    TRY(hipMemcpyAsync(&h[27], tst + 2, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    if (h[27] != quota) return NLP_ERR_DEVICE;
  } else if (ties > quota) {
    // canonical tie order: (u asc, w asc)
    TRY(wsget(ws, B_HP_TIEK1, ties, &tk1));
    TRY(wsget(ws, B_HP_TIEI1, ties, &ti1));
    const int vb = bits_for(g->span - 1);
    int shifts[8], np = 0;
    for (int b = 0; b < vb; b += 8) shifts[np++] = b;
    for (int b = 0; b < vb; b += 8) shifts[np++] = 32 + b;
    int which = 0;
    { nlp_status so = sort_pairs_os(g, tk0, ti0, tk1, ti1, ties, shifts, np, &which, st); if (so != NLP_OK) return so; }
    take_idx = which ? ti1 : ti0;
  }
  if (quota && !(ties > quota && 2 * svb <= 4 * TS_BITS))
    LAUNCH(k_hp_take, quota, st, take_idx, quota, above, ckey, cu, cw, cs, nk, nu, nw, ns);
  TRY(hipGetLastError());
  std::swap(ws.p[B_CKEY], ws.p[B_TKEY]); std::swap(ws.bytes[B_CKEY], ws.bytes[B_TKEY]);
  std::swap(ws.p[B_CU], ws.p[B_TU]); std::swap(ws.bytes[B_CU], ws.bytes[B_TU]);
  std::swap(ws.p[B_CW], ws.p[B_TW]); std::swap(ws.bytes[B_CW], ws.bytes[B_TW]);
  std::swap(ws.p[B_CS], ws.p[B_TS]); std::swap(ws.bytes[B_CS], ws.bytes[B_TS]);
  // three select histograms (4 B key each), the split (16 B in per candidate, 16 B out per kept)
  C.call_bytes += 28 * n + 16 * k;
  C.n = k;
  return NLP_OK;
}

// The held candidates straight to the caller's edges in the canonical order
// (score key desc, u asc, w asc): one record sort (es_sort).
// The canonical order of n links given as columns (u, w, score) written to
// `out` as records: one stable LSD sort of the records by
// (~score_key, u, w) (edgesort.hpp).  Digits that are the same for every
// record are skipped (one histogram read decides, read back with one sync).
// The look-back descriptors of the record passes: cleared when the buffer is
// new or regrown (size OR address) or the epochs run out, so no stale word can
// carry a live epoch.
nlp_status es_descs(nlp_graph* g, uint64_t ntiles, int P, uint64_t** desc, hipStream_t st) {
  Workspace& ws = g->ws;
  TRY(wsget(ws, B_ES_DESC, ntiles * 256, desc));
  if (ws.bytes[B_ES_DESC] != g->es_desc_bytes || (const void*)*desc != g->es_desc_ptr || g->es_epoch + P >= 0xffffull) {
    TRY(hipMemsetAsync(*desc, 0, ws.bytes[B_ES_DESC], st));
    g->es_desc_bytes = ws.bytes[B_ES_DESC];
    g->es_desc_ptr = *desc;
    g->es_epoch = 0;
  }
  return NLP_OK;
}

// The metrics whose score moves with deg w for a fixed (u, common count):
// Jaccard, Sorensen, Salton, Leicht-Holme-Newman.  Their runs of equal (rank,
// u) are short (C4 JAC H=16: none beyond 64 keys), so the two-level form
// pays; CN / AA / RA (the score of a u shared by every w with the same common
// neighbours) and HPI / HDI (c / deg u for every w on one side of deg u) have
// long runs (C4 H=16: CN 287,505 beyond 64 keys and 215 beyond 8192, AA
// 114,093 and 66): the whole sort there (11 ms against 60 / 31 ms).
bool es_runs_metric(int m) { return m == M_JAC || m == M_SOR || m == M_SAL || m == M_LHN; }

// The two-level order's run pass (edgesort.hpp k_es_runs, k_es_long; the very
// long runs by k_es_vgather, lsd8_keys and k_es_vscatter): `keys` (n K8 keys)
// sorted by (rank, u), every run of equal (rank, u) put in w order and the
// first nout written to `out` as edges.  `spare` (n keys) is free scratch.
nlp_status es_runs_order(nlp_graph* g, const float* rscore, const uint64_t* keys, uint64_t* spare, uint64_t n, int vb,
                         EdgeOut* out, uint64_t nout, hipStream_t st) {
  Workspace& ws = g->ws;
  const uint32_t rs = std::min<uint32_t>(std::max<uint32_t>(g->es_rs, 1), ER_RSMAX);
  const uint32_t lcap = std::min<uint32_t>(std::max<uint32_t>(g->es_lcap, 2), EL_CAPMAX);
  // a long run is longer than rs, a very long one than lcap: the lists' bounds
  const uint64_t lmax = n / (rs + 1) + 1, vmax = n / (lcap + 1) + 1;
  uint64_t* rb;  // [0] long runs, [1] very long runs, the long list, (start, length) pairs, the run table
  TRY(wsget(ws, B_ES_RUNS, 2 + lmax + 5 * vmax, &rb));
  uint64_t *lst = rb + 2, *vl = lst + lmax, *vt = vl + 2 * vmax;
  TRY(hipMemsetAsync(rb, 0, 16, st));
  const uint64_t ntl = (n + ER_TILE - 1) / ER_TILE;
  hipLaunchKernelGGL(k_es_runs, dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ntl, 2048))), dim3(ES_NT), 0,
                     st, rscore, keys, n, vb, out, nout, rs, lst, lmax, (unsigned long long*)rb);
  hipLaunchKernelGGL(k_es_long, dim3(512), dim3(EL_NT), 0, st, rscore, keys, n, vb, out, nout, lcap,
                     (const uint64_t*)lst, lmax, (const unsigned long long*)rb, vl, vmax, (unsigned long long*)(rb + 1));
  TRY(hipGetLastError());
  uint64_t hc[2] = {0, 0};
  TRY(hipMemcpyAsync(hc, rb, 16, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  if (hc[0] > lmax || hc[1] > vmax) return NLP_ERR_DEVICE;  // the lists' bounds are exact: never expected
  static const bool trace = getenv("NLP_TRACE_RUNS") && getenv("NLP_TRACE_RUNS")[0] == '1';
  if (trace)
    fprintf(stderr, "nlp runs: %llu keys, %llu runs beyond %u keys, %llu beyond %u\n", (unsigned long long)n,
            (unsigned long long)hc[0], rs, (unsigned long long)hc[1], lcap);
  if (hc[1] == 0) return NLP_OK;
  const uint64_t nv = hc[1];
  std::vector<uint64_t> pr(2 * nv), tab(3 * nv);
  TRY(hipMemcpyAsync(pr.data(), vl, 16 * nv, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  uint64_t tot = 0;
  for (uint64_t r = 0; r < nv; ++r) {
    tab[3 * r] = pr[2 * r];
    tab[3 * r + 1] = pr[2 * r + 1];
    tab[3 * r + 2] = tot;
    tot += pr[2 * r + 1];
  }
  if (tot > n) return NLP_ERR_DEVICE;
  TRY(hipMemcpyAsync(vt, tab.data(), 24 * nv, hipMemcpyHostToDevice, st));
  uint64_t* x1;
  TRY(wsget(ws, B_ES_TMP, tot, &x1));
  const unsigned gv = (unsigned)std::min<uint64_t>(nv, 4096);
  hipLaunchKernelGGL(k_es_vgather, dim3(gv), dim3(256), 0, st, keys, (const uint64_t*)vt, nv, vb, spare);
  TRY(hipGetLastError());
  // (run index, w): the runs keep their places and lengths, each in w order
  const int nb = vb + (nv > 1 ? bits_for(nv - 1) : 0);
  int shifts[ES_MAXP], np = 0;
  for (int b = 0; b < nb && np < ES_MAXP; b += 8) shifts[np++] = b;
  int which = 0;
  bool sorted = false;
  { nlp_status s = lsd8_keys(g, spare, x1, tot, shifts, np, &which, st, &sorted); if (s != NLP_OK) return s; }
  if (!sorted) return NLP_ERR_INVALID;
  hipLaunchKernelGGL(k_es_vscatter, dim3(gv), dim3(256), 0, st, rscore, (const uint64_t*)(which ? x1 : spare), keys,
                     (const uint64_t*)vt, nv, vb, out, nout);
  TRY(hipGetLastError());
  TRY(hipStreamSynchronize(st));  // `tab` is read by the copy above
  return NLP_OK;
}

// es_sort over rank-compressed 8-byte keys (edgesort.hpp k_es_dkeys, k_es_hist8,
// k_es_pass8).  *done = false when the call does not qualify (too many distinct
// score keys, a NaN or zero score, too many key bits): nothing was written.
// ckey != nullptr: the input is an UNPRUNED buffer of n candidates whose score
// keys are ckey; only those >= kmin are sorted, and the first nout of them (in
// canonical order) are written -- the prune's split and tie selection folded
// into the sort (the canonical tie rule is the sort order itself).
nlp_status es_sort8(nlp_graph* g, const uint32_t* cu, const uint32_t* cw, const float* cs, uint64_t n, EdgeOut* out,
                    hipStream_t st, uint64_t* bytes, bool* done, const uint32_t* ckey = nullptr, uint32_t kmin = 0,
                    uint64_t nout = UINT64_MAX, bool* runs = nullptr, bool runs_ok = false) {
  *done = false;
  Workspace& ws = g->ws;
  const int vb = std::max(1, bits_for(g->span - 1));
  if (2 * vb > 63) return NLP_OK;
  // [ES_DCAP] set, [4] counts, then the rank scores (f32)
  uint32_t* dset;
  const uint64_t words = ES_DCAP + 4 + ES_DMAX;
  TRY(wsget(ws, B_ES_SET, words, &dset));
  uint32_t* dcnt = dset + ES_DCAP;
  float* rscore = (float*)(dcnt + 4);
  TRY(hipMemsetAsync(dset, 0, (ES_DCAP + 4) * 4, st));
  hipLaunchKernelGGL(k_es_dkeys, dim3((unsigned)std::min<uint64_t>((n + ES_NT * 8 - 1) / (ES_NT * 8), 2048)), dim3(ES_NT), 0, st,
                     cs, n, dset, dcnt, ckey, kmin);
  TRY(hipGetLastError());
  std::vector<uint32_t> hs(ES_DCAP + 4);
  TRY(hipMemcpyAsync(hs.data(), dset, (ES_DCAP + 4) * 4, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  const uint32_t D = hs[ES_DCAP], over = hs[ES_DCAP + 1];
  if (over || D == 0 || D > ES_DMAX) return NLP_OK;
  std::vector<uint32_t> keys;
  keys.reserve(D);
  for (uint32_t i = 0; i < ES_DCAP; ++i)
    if (hs[i]) keys.push_back(hs[i] - 1u);
  if (keys.size() != D) return NLP_OK;
  for (uint32_t k : keys)
    if (k == 0u || k == 0x80000000u) return NLP_OK;  // NaN / zero: several bit patterns behind one key
  const int rb = D > 1 ? bits_for(D - 1) : 0;
  if (rb + 2 * vb > 64 || n >= (1ull << 32)) return NLP_OK;  // 32-bit range offsets
  const uint64_t n_in = n;
  std::sort(keys.begin(), keys.end(), std::greater<uint32_t>());  // rank 0 = the highest score
  std::vector<float> hsc(D);
  for (uint32_t r = 0; r < D; ++r) {
    const uint32_t k = keys[r];
    const uint32_t b = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;  // score_key's inverse
    memcpy(&hsc[r], &b, 4);
  }
  TRY(hipMemcpyAsync(rscore, hsc.data(), D * 4, hipMemcpyHostToDevice, st));
  uint64_t *k0 = nullptr, *k1 = nullptr;
  if (ckey) {  // the kept candidates' keys, compacted: the sort's n is their count
    TRY(wsget(ws, B_ES_K0, n, &k0));
    unsigned long long* kc = (unsigned long long*)(dcnt + 2);  // zeroed with the set
    hipLaunchKernelGGL(k_es_keep8, dim3((unsigned)std::min<uint64_t>((n + ES_NT * 8 - 1) / (ES_NT * 8), 2048)),
                       dim3(ES_NT), 0, st, ckey, cu, cw, n, kmin, vb, (const float*)rscore, D, k0, kc);
    TRY(hipGetLastError());
    unsigned long long kept = 0;
    TRY(hipMemcpyAsync(&kept, kc, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    if (kept < std::min<uint64_t>(nout, n) || kept > n) return NLP_ERR_DEVICE;
    n = kept;
  }
  // the keys (and the first pass's range counts) in one read; ranges of tpw
  // tiles, one workgroup each
  const Es8Shape sh8 = es8_shape(g);
  const uint64_t ntiles = (n + sh8.tile - 1) / sh8.tile;
  uint32_t G = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({ntiles, (uint64_t)sh8.occ, (uint64_t)ES8_GMAX}));
  const uint32_t tpw = (uint32_t)((ntiles + G - 1) / G);
  G = (uint32_t)((ntiles + tpw - 1) / tpw);  // every range non-empty
  // the two-level form (edgesort.hpp k_es_runs): passes over the (rank, u)
  // bits only, then the runs of equal (rank, u) put in w order in place -- the
  // run pass stands in for the last pass (both read the keys and write the
  // edges), so it pays from two passes saved
  const int Pf = std::max(1, (rb + 2 * vb + 7) / 8), Ph = std::max(1, (rb + vb + 7) / 8);
  const bool two = g->es_runs == 2 || (g->es_runs == 1 && runs_ok && Ph + 2 <= Pf);
  const int P = two ? Ph : Pf, sh0 = two ? vb : 0;
  {
    static const bool trace = getenv("NLP_TRACE_RUNS") && getenv("NLP_TRACE_RUNS")[0] == '1';
    if (trace)
      fprintf(stderr, "nlp order: %llu keys, %u scores (%d rank bits), %d id bits, %d passes (%d without runs), "
              "%d-thread passes\n", (unsigned long long)n, D, rb, vb, P, Pf, sh8.nt);
  }
  uint32_t* hw;  // [P][256] digit totals
  TRY(wsget(ws, B_ES_HIST, (uint64_t)ES_MAXP * 256 + ES_MAXP + 4, &hw));
  TRY(hipMemsetAsync(hw, 0, (uint64_t)P * 256 * 4, st));
  uint32_t* cnt;  // [256][G] range counts, then [256][G] offsets
  TRY(wsget(ws, B_ES_CNT, (uint64_t)2 * 256 * G, &cnt));
  uint32_t* offs = cnt + (uint64_t)256 * G;
  if (!ckey) TRY(wsget(ws, B_ES_K0, n, &k0));
  if (two || P > 1) TRY(wsget(ws, B_ES_K1, n, &k1));
  if (ckey) {
    hipLaunchKernelGGL(k_es_cnt8, dim3(G), dim3(ES_NT), 0, st, (const uint64_t*)k0, n, sh0, cnt, hw, tpw, G,
                       sh8.tile);
  } else {
    hipLaunchKernelGGL(k_es_hist8, dim3(G), dim3(ES_NT), 0, st, cu, cw, cs, n, vb, (const float*)rscore, D, hw, k0,
                       cnt, tpw, G, sh0, sh8.tile);
  }
  TRY(hipGetLastError());
  // scores (4 B), columns in and keys out (20 B), every later pass's count
  // read (8 B), every pass but the last 8 in and out, the last 8 in, 12 out;
  // filtered: keys of every candidate (8 B), the kept ones' columns (8 B) and
  // keys out (8 B), the first pass's count read (8 B); two-level: P passes
  // of keys, the run pass 8 in, 12 out
  const uint64_t nw = std::min<uint64_t>(nout, n);
  if (bytes)
    *bytes += (ckey ? 8 * n_in + 24 * n : 24 * n) + 24 * n * (uint64_t)(two ? P : P - 1) + 8 * n + 12 * nw;
  const uint64_t* src = k0;  // k_es_hist8 wrote every key
  for (int r = 0; r < P; ++r) {
    uint64_t* dst = (r & 1) ? k0 : k1;
    const int sh = sh0 + 8 * r;
    if (r > 0) {  // this pass's range counts: one read of its input
      hipLaunchKernelGGL(k_es_cnt8, dim3(G), dim3(ES_NT), 0, st, src, n, sh, cnt, hw + r * 256, tpw, G, sh8.tile);
      TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(k_es_off8, dim3(256), dim3(ES8_GMAX), 0, st, (const uint32_t*)cnt,
                       (const uint32_t*)(hw + r * 256), G, offs);
    TRY(hipGetLastError());
    es8_pass(sh8, r == P - 1 && !two, G, st, (const float*)rscore, src, dst, out, n, vb, sh, offs, tpw, nw);
    TRY(hipGetLastError());
    src = dst;
  }
  if (two) {
    nlp_status s = es_runs_order(g, (const float*)rscore, src, src == k0 ? k1 : k0, n, vb, out, nw, st);
    if (s != NLP_OK) return s;
    if (runs) *runs = true;
  }
  *done = true;
  return NLP_OK;
}

// try8 = false: the caller already knows the keys refuse the 8-byte order.
// *route (may be null): NLP_ORDER_SORT8 or NLP_ORDER_SORT12, the sort that ran.
nlp_status es_sort(nlp_graph* g, const uint32_t* cu, const uint32_t* cw, const float* cs, uint64_t n, EdgeOut* out,
                   hipStream_t st, uint64_t* bytes = nullptr, bool try8 = true, uint32_t* route = nullptr,
                   int metric = -1) {
  if (n == 0) return NLP_OK;
  if (try8 && ((n >= ES8_MIN && g->es_k8 == 1) || g->es_k8 == 2)) {
    bool done = false, runs = false;
    nlp_status s = es_sort8(g, cu, cw, cs, n, out, st, bytes, &done, nullptr, 0, UINT64_MAX, &runs,
                            es_runs_metric(metric));
    if (s != NLP_OK) return s;
    if (done) {
      if (route) *route = NLP_ORDER_SORT8 | (runs ? NLP_ORDER_RUNS : 0u);
      return NLP_OK;
    }
  }
  if (route) *route = NLP_ORDER_SORT12;
  Workspace& ws = g->ws;
  const int vb = std::max(1, bits_for(g->span - 1));
  const int npass = (32 + 2 * vb + 7) / 8;
  if (npass > ES_MAXP || n >= ES_AGG) return NLP_ERR_INVALID;
  uint32_t* hw;  // [npass * 256] histograms, [ES_MAXP] tickets, error word
  TRY(wsget(ws, B_ES_HIST, (uint64_t)ES_MAXP * 256 + ES_MAXP + 4, &hw));
  uint32_t* tick = hw + ES_MAXP * 256;
  uint32_t* err = tick + ES_MAXP;
  TRY(hipMemsetAsync(hw, 0, ((uint64_t)ES_MAXP * 256 + ES_MAXP + 4) * 4, st));
  hipLaunchKernelGGL(k_es_hist, dim3((unsigned)std::min<uint64_t>((n + ES_NT - 1) / ES_NT, 2048)), dim3(ES_NT), 0, st,
                     cu, cw, cs, n, vb, npass, hw);
  TRY(hipGetLastError());
  std::vector<uint32_t> h((size_t)npass * 256);
  TRY(hipMemcpyAsync(h.data(), hw, h.size() * 4, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  int run[ES_MAXP], P = 0;
  for (int p = 0; p < npass; ++p) {
    uint32_t mx = 0;
    for (int d = 0; d < 256; ++d) mx = std::max(mx, h[(size_t)p * 256 + d]);
    if (mx < n) run[P++] = p;
  }
  if (bytes) *bytes += 12 * n + 24 * n * (uint64_t)std::max(P, 1);  // histogram read + every pass in and out
  if (P == 0) {
    LAUNCH(k_es_copy, n, st, cu, cw, cs, n, out);
    return hipGetLastError() == hipSuccess ? NLP_OK : NLP_ERR_DEVICE;
  }
  const uint64_t ntiles = (n + (uint64_t)ES_NT * ES_IPT - 1) / ((uint64_t)ES_NT * ES_IPT);
  uint64_t* desc;
  EdgeOut* tmp = nullptr;
  { nlp_status s = es_descs(g, ntiles, P, &desc, st); if (s != NLP_OK) return s; }
  if (P > 1) TRY(wsget(ws, B_ES_TMP, n, &tmp));
  const unsigned gr = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ntiles, g->occ_es));
  const EdgeOut* src = nullptr;
  for (int r = 0; r < P; ++r) {
    EdgeOut* dst = ((P - 1 - r) & 1) ? tmp : out;  // the last pass writes `out`
    const uint64_t ep = ++g->es_epoch;
    if (r == 0)
      hipLaunchKernelGGL(k_es_pass<true>, dim3(gr), dim3(ES_NT), 0, st, cu, cw, cs, (const EdgeOut*)nullptr, dst, n, vb,
                         8 * run[r], (const uint32_t*)(hw + run[r] * 256), desc, tick + r, ep, err);
    else
      hipLaunchKernelGGL(k_es_pass<false>, dim3(gr), dim3(ES_NT), 0, st, (const uint32_t*)nullptr,
                         (const uint32_t*)nullptr, (const float*)nullptr, src, dst, n, vb, 8 * run[r],
                         (const uint32_t*)(hw + run[r] * 256), desc, tick + r, ep, err);
    TRY(hipGetLastError());
    src = dst;
  }
  uint32_t herr = 0;
  TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  return herr ? NLP_ERR_DEVICE : NLP_OK;  // a look-back gave up (never expected)
}

nlp_status hp_final_order(nlp_graph* g, Cands& C, EdgeOut* d_out, hipStream_t st) {
  if (C.n == 0) return NLP_OK;
  if (C.keep) {  // the last prune folded into the 8-byte order
    bool done = false, runs = false;
    Workspace& ws = g->ws;
    nlp_status s = es_sort8(g, (const uint32_t*)ws.p[B_CU], (const uint32_t*)ws.p[B_CW], (const float*)ws.p[B_CS], C.n,
                            d_out, st, &C.call_bytes, &done, (const uint32_t*)ws.p[B_CKEY], C.kmin, C.keep, &runs,
                            es_runs_metric(C.metric));
    if (s != NLP_OK) return s;
    const uint64_t keep = C.keep;
    C.keep = 0;
    if (done) {
      C.n = keep;
      C.route = NLP_ORDER_FOLD8 | (runs ? NLP_ORDER_RUNS : 0u);
      return NLP_OK;
    }
    // the keys do not qualify (too many distinct scores, ...): prune, then the
    // 12-byte order (the kept keys are a subset of the refused ones)
    uint32_t kth = 0;
    s = hp_prune(g, C, keep, C.cap, &kth, st);
    if (s != NLP_OK) return s;
    s = es_sort(g, (const uint32_t*)g->ws.p[B_CU], (const uint32_t*)g->ws.p[B_CW], (const float*)g->ws.p[B_CS], C.n,
                d_out, st, &C.call_bytes, false);
    C.route = NLP_ORDER_FOLD_REFUSED;
    return s;
  }
  return es_sort(g, (const uint32_t*)g->ws.p[B_CU], (const uint32_t*)g->ws.p[B_CW], (const float*)g->ws.p[B_CS], C.n,
                 d_out, st, &C.call_bytes, true, &C.route, C.metric);
}

// Estimated wedges (w > u) of a call: sum over surviving v of deg(v)^2 / 2,
// scaled to the source range.
double hp_estimate(const nlp_graph* g, const Params& p) {
  const uint64_t S = g->span;
  const uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S);
  double w = 0;
  for (size_t d = 1; d < g->deg_hist.size(); ++d)
    if (p.H == 0 || d <= p.H) w += (double)d * (double)d * (double)g->deg_hist[d];
  if (p.H == 0 || p.H > DCAP) w += (double)g->big_deg2;  // upper bound for DCAP < H
  return S ? 0.5 * w * (double)(ub - ua) / (double)S : 0.0;
}

// The hub pass over a chunk's bin-2 and bin-3 rows (hashpath.hpp, k_hh_*).
// *done = false: the chunk's hub wedges exceed the scratch (the caller runs
// k_hp_part instead; nothing was emitted).
nlp_status run_hub(nlp_graph* g, const HpArgs& a, const uint32_t* l2, uint64_t n2, const uint32_t* l3, uint64_t n3,
                   const uint64_t* wu, uint64_t ua, bool custom, uint64_t* scan, uint32_t* queue, bool* done,
                   hipStream_t st, uint64_t* hub_wedges = nullptr) {
  Workspace& ws = g->ws;
  *done = false;
  const uint64_t nh = n2 + n3;
  uint32_t* hr;    // u, shift, P, items: 4 x nh
  uint64_t* pre;   // bucket prefix [nh + 1], item prefix [nh + 1], first-hop count [nh], first-hop prefix [nh + 1]
  TRY(wsget(ws, B_HH_ROWS, 4 * nh, &hr));
  TRY(wsget(ws, B_HH_PRE, 4 * (nh + 1), &pre));
  uint32_t *hr_u = hr, *hr_shift = hr + nh, *hr_p = hr + 2 * nh, *hr_items = hr + 3 * nh;
  uint64_t *bbase = pre, *ibase = pre + nh + 1, *hr_nf = pre + 2 * (nh + 1), *fbase = pre + 3 * (nh + 1);
  LAUNCH(k_hh_rows, nh, st, a, l2, n2, l3, n3, wu, ua, hr_u, hr_shift, hr_p, hr_items, hr_nf, g->hh_bw);
  TRY(hipGetLastError());
  // first hops -> the prefix of their lists' parts above u (k_hh_fpre), then the
  // buckets and items of every row from the wedges it really enumerates (k_hh_items)
  TRY(scan_ws<uint64_t>(ws, B_SCAN, hr_nf, nh, fbase, fbase + nh, st));
  TRY(hipMemcpyAsync(&g->host_small[51], fbase + nh, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  const uint64_t NF = g->host_small[51];
  if (NF == 0) {
    *done = true;
    return NLP_OK;
  }
  uint64_t* fp;
  TRY(wsget(ws, B_HH_FP, std::max<uint64_t>(NF, 1), &fp));
  hipLaunchKernelGGL(k_hh_fpre, dim3((unsigned)std::min<uint64_t>(nh, 4096)), dim3(HH_NT), 0, st, a, nh,
                     (const uint32_t*)hr_u, (const uint64_t*)hr_nf, (const uint64_t*)fbase, fp);
  LAUNCH(k_hh_items, nh, st, a, nh, (const uint32_t*)hr_u, (const uint64_t*)hr_nf, (const uint64_t*)fbase,
         (const uint64_t*)fp, hr_shift, hr_p, hr_items, g->hh_bw);
  TRY(hipGetLastError());
  TRY(scan_ws<uint32_t>(ws, B_SCAN, hr_p, nh, bbase, bbase + nh, st));
  TRY(scan_ws<uint32_t>(ws, B_SCAN, hr_items, nh, ibase, ibase + nh, st));
  TRY(hipMemcpyAsync(&g->host_small[48], bbase + nh, 8, hipMemcpyDeviceToHost, st));
  TRY(hipMemcpyAsync(&g->host_small[49], ibase + nh, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  const uint64_t NB = g->host_small[48], NI = g->host_small[49];
  if (NB == 0 || NI == 0) {
    *done = true;
    return NLP_OK;
  }
  if (NI > 0x7fffffffull) return NLP_OK;
  uint32_t* maps;  // brow [NB]
  uint32_t* bc;    // bcnt [NB], bcur [NB]
  uint64_t *boff, *xs;
  TRY(wsget(ws, B_HH_MAPS, NB, &maps));
  TRY(wsget(ws, B_HH_BCNT, 2 * NB, &bc));
  TRY(wsget(ws, B_HH_BOFF, NB + 1, &boff));
  TRY(wsget(ws, B_HH_XS, NB, &xs));
  uint32_t *brow = maps, *bcnt = bc, *bcur = bc + NB;
  TRY(hipMemsetAsync(bc, 0, 2 * NB * 4, st));
  LAUNCH(k_hh_maps, nh, st, a, nh, (const uint32_t*)hr_u, (const uint32_t*)hr_shift, (const uint32_t*)hr_p,
         (const uint64_t*)bbase, (const uint32_t*)hr_items, (const uint64_t*)ibase, brow, (uint32_t*)nullptr);
  LAUNCH(k_hh_xstart, NB, st, a, NB, (const uint32_t*)brow, (const uint32_t*)hr_u, (const uint32_t*)hr_shift,
         (const uint64_t*)bbase, xs);
  TRY(hipGetLastError());
  if (custom)
    hipLaunchKernelGGL((k_hh_enum<false, true>), dim3((unsigned)NI), dim3(HH_NT), 0, st, a, nh, (const uint32_t*)hr_u,
                       (const uint32_t*)hr_shift, (const uint32_t*)hr_p, (const uint64_t*)bbase, (const uint64_t*)ibase,
                       (const uint64_t*)fbase, (const uint64_t*)fp, bcnt, (const uint64_t*)nullptr, (uint32_t*)nullptr,
                       (uint32_t*)nullptr, (uint32_t*)nullptr);
  else
    hipLaunchKernelGGL((k_hh_enum<false, false>), dim3((unsigned)NI), dim3(HH_NT), 0, st, a, nh, (const uint32_t*)hr_u,
                       (const uint32_t*)hr_shift, (const uint32_t*)hr_p, (const uint64_t*)bbase, (const uint64_t*)ibase,
                       (const uint64_t*)fbase, (const uint64_t*)fp, bcnt, (const uint64_t*)nullptr, (uint32_t*)nullptr,
                       (uint32_t*)nullptr, (uint32_t*)nullptr);
  TRY(hipGetLastError());
  // the buckets can outnumber the chunk's rows (the caller's scan scratch is
  // sized for those): a scratch of their own
  uint64_t* bscan;
  TRY(wsget(ws, B_HH_SCAN, scan_scratch_words(NB + 1) + 16, &bscan));
  TRY(scan_ws<uint32_t>(ws, B_HH_SCAN, bcnt, NB, boff, boff + NB, st));
  TRY(hipMemcpyAsync(&g->host_small[50], boff + NB, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  const uint64_t tot = g->host_small[50];
  if (hub_wedges) *hub_wedges += tot;
  TRY(hipMemsetAsync(bcur, 0, NB * 4, st));
  const uint64_t words = (uint64_t)g->hp_gp * g->hp_scap * 2;  // u32 words of the k_hp_part scratch
  const uint64_t capw = custom ? words / 2 : words;
  if (tot > capw || tot > 0xffffffffull) return NLP_OK;  // k_hp_part for this chunk
  uint32_t* sw = g->hp_scratch;
  uint32_t* sv = custom ? g->hp_scratch + capw : nullptr;
  if (custom)
    hipLaunchKernelGGL((k_hh_enum<true, true>), dim3((unsigned)NI), dim3(HH_NT), 0, st, a, nh, (const uint32_t*)hr_u,
                       (const uint32_t*)hr_shift, (const uint32_t*)hr_p, (const uint64_t*)bbase, (const uint64_t*)ibase,
                       (const uint64_t*)fbase, (const uint64_t*)fp, bcnt, (const uint64_t*)boff, bcur, sw, sv);
  else
    hipLaunchKernelGGL((k_hh_enum<true, false>), dim3((unsigned)NI), dim3(HH_NT), 0, st, a, nh, (const uint32_t*)hr_u,
                       (const uint32_t*)hr_shift, (const uint32_t*)hr_p, (const uint64_t*)bbase, (const uint64_t*)ibase,
                       (const uint64_t*)fbase, (const uint64_t*)fp, bcnt, (const uint64_t*)boff, bcur, sw, sv);
  TRY(hipGetLastError());
  // accumulation items (k_hh_plan, k_hh_group): a bucket, or a w-range of a heavy bucket
  // count metrics: 4096-entry tables by default (C5 range: 47.7 -> 41.9 ms against 8192 entries, two
  // workgroups per CU more; 2048 entries split too many buckets: 176 ms)
  const int tl = std::min(custom ? HH_TL - 1 : HH_TL, g->hh_tl ? g->hh_tl : HH_TLC);
  // AA / RA: sort-mode items (at most HH_SCAP wedges each, keys need w, v < 2^26)
  const uint32_t wcap = custom && g->hh_sort && g->span <= (1ull << 26) ? g->hh_scap : 0u;
  // heavy buckets hold more than `half` wedges each; their groups close past
  // `half` wedges, so a heavy bucket of n wedges gives at most 2 n / half + 2
  // items (single bins beyond a group included)
  const uint32_t dw = custom ? 0u : std::min<uint32_t>(g->hh_dw, 2u << tl);  // direct counters: counts only,
                                                                             // within the table's two words
  const uint64_t half = wcap ? wcap : (1ull << (tl - 1));
  const uint64_t hcap = tot / half + 1;
  const uint64_t cap = NB + 4 * (tot / half) + 2 * hcap + 1024;
  const uint64_t gwords = HH_BPS * (tot / HH_SEG + hcap + 1);  // bins: HH_BPS per segment
  HhItem* items;
  uint64_t* hv;  // the packed heavy counter, then the heavy buckets
  uint64_t* gh;
  TRY(wsget(ws, B_HH_SITEM, cap * sizeof(HhItem) / 8 + 1, (uint64_t**)&items));
  TRY(wsget(ws, B_HH_HEAVY, 1 + hcap * sizeof(HhHeavy) / 8, &hv));
  TRY(wsget(ws, B_HH_GHIST, gwords + 2, &gh));  // bins, then the item cursors
  uint32_t* pw;  // the heavy buckets' wedges partitioned by item (and v for AA / RA): bucket offsets as in sw
  TRY(wsget(ws, B_HH_PART, (custom ? 2 * tot : tot) + 2, &pw));
  uint32_t* pv = custom ? pw + tot : nullptr;
  uint32_t* gcur = (uint32_t*)gh + gwords;
  HhHeavy* heavy = (HhHeavy*)(hv + 1);
  unsigned long long* hctr = (unsigned long long*)hv;
  uint32_t* nitems = queue + 1;
  TRY(hipMemsetAsync(queue, 0, 8, st));
  TRY(hipMemsetAsync(hv, 0, 8, st));
  LAUNCH(k_hh_plan, NB, st, a, NB, (const uint32_t*)brow, (const uint32_t*)hr_u, (const uint32_t*)hr_shift,
         (const uint32_t*)hr_p, (const uint64_t*)bbase, (const uint64_t*)boff, (const uint64_t*)xs,
         (const uint32_t*)bcnt, tl, items, nitems, heavy, hctr, hcap, (uint32_t*)gh, wcap, dw);
  hipLaunchKernelGGL(k_hh_hist, dim3((unsigned)std::min<uint64_t>(tot / HH_SEG + hcap, 4096)), dim3(HH_NT), 0, st, a,
                     (const HhHeavy*)heavy, (const unsigned long long*)hctr, hcap, (const uint64_t*)boff,
                     (const uint32_t*)sw, (uint32_t*)gh);
  hipLaunchKernelGGL(k_hh_group, dim3((unsigned)std::min<uint64_t>(hcap, 1024)), dim3(HH_NT), 0, st, a,
                     (const HhHeavy*)heavy, (const unsigned long long*)hctr, hcap, (uint32_t*)gh, gcur,
                     (const uint64_t*)boff, tl, items, nitems, cap, wcap, dw);
  hipLaunchKernelGGL(k_hh_part, dim3((unsigned)std::min<uint64_t>(tot / HH_SEG + hcap, 4096)), dim3(HH_NT), 0, st, a,
                     (const HhHeavy*)heavy, (const unsigned long long*)hctr, hcap, (const uint64_t*)boff,
                     (const uint32_t*)sw, (const uint32_t*)sv, (const uint32_t*)gh, gcur, pw, pv);
  TRY(hipGetLastError());
  // persistent workgroups over the item queue: the table's LDS decides how many fit a CU
  const unsigned gr = (unsigned)((custom || tl >= 13 ? 4 : 8) * (uint64_t)g->hp_gp);
  HpArgs ah = a;  // NLP_TRACE_HUB=1: the sort mode's phase ticks into the chunk counters' small[56, 60)
  static const bool trace_hub = getenv("NLP_TRACE_HUB") && getenv("NLP_TRACE_HUB")[0] == '1';
  ah.ph = trace_hub ? a.ctr + 56 : nullptr;
#define NLP_HH_ACCUM(CU, TLC)                                                                                 \
  hipLaunchKernelGGL((k_hh_accum<CU, TLC>), dim3(gr), dim3(HH_NT), 0, st, ah, (const HhItem*)items,           \
                     (const uint32_t*)nitems, (const uint32_t*)sw, (const uint32_t*)sv, (const uint32_t*)pw, \
                     (const uint32_t*)pv, queue, (int)wcap, cap)
  if (custom) NLP_HH_ACCUM(true, HH_TL);
  else if (tl >= 13) NLP_HH_ACCUM(false, 13);
  else if (tl == 12) NLP_HH_ACCUM(false, 12);
  else NLP_HH_ACCUM(false, 11);
#undef NLP_HH_ACCUM
  TRY(hipGetLastError());
  *done = true;
  return NLP_OK;
}

nlp_status run_path3(nlp_graph* g, const Params& p, Cands& C, uint32_t* nchunks, hipStream_t st) {
  Workspace& ws = g->ws;
  const uint64_t S = g->span;
  const uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S), nU = ub - ua;
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  uint64_t k = p.max_edges;
  *nchunks = 0;
  if (nU == 0 || g->nnz == 0) return NLP_OK;
  { nlp_status s0 = hp_alloc_scratch(g); if (s0 != NLP_OK) return s0; }
  uint64_t *wu, *pos, *small;
  TRY(wsget(ws, B_HP_WU, nU + 1, &wu));
  TRY(wsget(ws, B_HP_POS, nU + 1, &pos));
  TRY(wsget(ws, B_HP_SMALL, 72, &small));  // [64, 68): NLP_TRACE_BATCH phase ticks
  uint64_t* scan;
  TRY(wsget(ws, B_SCAN, scan_scratch_words(nU + 1) + 16, &scan));
  // small: [0,8) chunk counters, [8] tau, [16,24) bounds, [24,28) list sizes, [32..] prune scratch
  const GraphView gv = view_of(g, p.metric, p.maxf2);
  uint64_t* s_soff = nullptr;  // survivor lists S(u) of the range (small H), see k_hp_surv_lists / k_hp_dcls_*
  uint32_t* s_skeys = nullptr;
  bool s_sorted = false;       // S(u) in N(u)'s order (degree-class compaction)
  uint64_t* s_sdo = nullptr;   // packed S(u) entries (deg v, off[v]) of the degree-class lists
  const uint64_t b1max = custom ? HP_BT / 4 : HP_B1_MAX;  // the largest W(u) of bin 1
  const uint32_t* s_scn = nullptr;  // |S(u)| when S(u) are prefixes of the class-ordered short lists
  uint64_t* scan2 = nullptr;
  {
    TRY(hipMemsetAsync(wu, 0, nU * 8, st));
    TRY(hipMemcpyAsync(&g->host_small[8], g->off + ua, 8, hipMemcpyDeviceToHost, st));
    TRY(hipMemcpyAsync(&g->host_small[9], g->off + ub, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    const uint64_t e0 = g->host_small[8], e1 = g->host_small[9];
    // small H: W(u) from the survivors' in-edges (P_H atomics) when that is well below the range's entries
    uint64_t p_h = ~0ull;
    if (p.H >= 1 && p.H <= DCAP && g->vbydeg && !g->deg_hist.empty()) {
      p_h = 0;
      for (uint32_t d = 1; d <= p.H; ++d) p_h += (uint64_t)d * g->deg_hist[d];
    }
    bool one_done = false;
    if (g->sl_off && !custom && g->hp_dcls && p.H >= 1 && p.H <= g->sl_cap) {
      // count metrics: S(u) = the prefix of u's class-ordered short list (deg v <= H); only the
      // prefixes' lengths and W+(u) are found (hashpath.hpp k_sl_count)
      uint32_t* scnt;
      TRY(wsget(ws, B_HP_SCNT, nU, &scnt));
      hipLaunchKernelGGL(k_sl_rows, dim3(grid_full(nU)), dim3(NT), 0, st, (const uint64_t*)g->sl_off,
                         (const uint8_t*)g->sl_cls, (const uint32_t*)g->sl_pn, p.H, ua, nU, scnt,
                         (unsigned long long*)wu);
      TRY(hipGetLastError());
      s_soff = g->sl_off + ua;
      s_scn = scnt;
      s_skeys = g->sl_keys;
      s_sdo = g->sl_sdo;
      s_sorted = false;
      one_done = true;
    }
    if (one_done) {
    } else if (g->dcls && g->hp_dcls && g->drank && p.H >= 1 &&
        p.H <= HP_DCLS_MAX && e1 > e0 && g->nnz < (1ull << HP_SDO_SH)) {
      // count, place, gather (hashpath.hpp k_dc_*)
      const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE, nt = t1 - t0;
      uint32_t *scnt, *tcn;
      uint64_t* tpre;
      TRY(wsget(ws, B_HP_SCNT, nU, &scnt));
      TRY(wsget(ws, B_HP_SOFF, nU + 1, &s_soff));
      TRY(wsget(ws, B_HP_TCNT, nt, &tcn));
      TRY(wsget(ws, B_HP_TPRE, nt + 1, &tpre));
      const unsigned gt = (unsigned)std::min<uint64_t>((nt + NWAVE - 1) / NWAVE, 16384);
      uint8_t* smask;
      TRY(wsget(ws, B_HP_SMASK, nt * 64, &smask));
      hipLaunchKernelGGL(k_dc_count, dim3(gt), dim3(NT), 0, st, (const uint8_t*)g->dcls, p.H, e0, e1, tcn, smask);
      TRY(hipGetLastError());
      TRY(wsget(ws, B_SCAN2, scan_scratch_words(nt) + 16, &scan2));
      TRY(scan_ws<uint32_t>(ws, B_SCAN2, tcn, nt, tpre, tpre + nt, st));
      TRY(hipMemcpyAsync(&g->host_small[10], tpre + nt, 8, hipMemcpyDeviceToHost, st));
      TRY(hipStreamSynchronize(st));
      const uint64_t ns = g->host_small[10];
      uint64_t* se;
      uint32_t* sr;
      TRY(wsget(ws, B_HP_SE, std::max<uint64_t>(ns, 1), &se));
      TRY(wsget(ws, B_HP_SR, std::max<uint64_t>(ns, 1), &sr));
      TRY(wsget(ws, B_HP_SKEYS, std::max<uint64_t>(ns, 1), &s_skeys));
      TRY(wsget(ws, B_HP_SDO, std::max<uint64_t>(ns, 1), &s_sdo));
      hipLaunchKernelGGL(k_dc_place, dim3(gt), dim3(NT), 0, st, gv, (const uint8_t*)smask, ua, nU, e0, e1,
                         (const uint32_t*)g->tile_row, (const uint64_t*)tpre, se, sr);
      if (ns)
        hipLaunchKernelGGL(k_dc_gather, dim3((unsigned)std::min<uint64_t>((ns + NT - 1) / NT, 65536)), dim3(NT), 0, st,
                           gv, (const uint8_t*)g->dcls, (const uint8_t*)g->drank, (const uint64_t*)se,
                           (const uint32_t*)sr, ns, s_skeys, s_sdo, (unsigned long long*)wu);
      TRY(hipGetLastError());
      LAUNCH(k_hp_unpack, nU, st, (unsigned long long*)wu, scnt, nU);
      TRY(hipGetLastError());
      TRY(scan_ws<uint32_t>(ws, B_SCAN, scnt, nU, s_soff, s_soff + nU, st));
      s_sorted = true;
      one_done = true;
    }
    if (one_done) {
    } else if (g->dcls && g->hp_dcls && p.H >= 1 && p.H <= HP_DCLS_MAX && e1 > e0) {
      // the survivor lists S(u) as the compaction of the range's entries by
      // degree class (sorted, no atomics; hashpath.hpp k_hp_dcls_*)
      const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE, nt = t1 - t0;
      uint32_t *scnt, *tcn;
      uint64_t* tpre;
      TRY(wsget(ws, B_HP_SCNT, nU, &scnt));
      TRY(wsget(ws, B_HP_SOFF, nU + 1, &s_soff));
      TRY(wsget(ws, B_HP_TCNT, nt, &tcn));
      TRY(wsget(ws, B_HP_TPRE, nt + 1, &tpre));
      const unsigned gt = (unsigned)std::min<uint64_t>((nt + NWAVE - 1) / NWAVE, 16384);
      hipLaunchKernelGGL(k_hp_dcls_rows8, dim3(gt), dim3(NT), 0, st, gv, (const uint8_t*)g->dcls, p.H, ua, nU, e0, e1,
                         (const uint32_t*)g->tile_row, (unsigned long long*)wu, tcn);
      TRY(hipGetLastError());
      LAUNCH(k_hp_unpack, nU, st, (unsigned long long*)wu, scnt, nU);
      TRY(hipGetLastError());
      TRY(scan_ws<uint32_t>(ws, B_SCAN, scnt, nU, s_soff, s_soff + nU, st));
      TRY(wsget(ws, B_SCAN2, scan_scratch_words(nt) + 16, &scan2));
      TRY(scan_ws<uint32_t>(ws, B_SCAN2, tcn, nt, tpre, tpre + nt, st));
      TRY(hipMemcpyAsync(&g->host_small[10], s_soff + nU, 8, hipMemcpyDeviceToHost, st));
      TRY(hipStreamSynchronize(st));
      TRY(wsget(ws, B_HP_SKEYS, std::max<uint64_t>(g->host_small[10], 1), &s_skeys));
      if (g->nnz < (1ull << HP_SDO_SH)) {
        TRY(wsget(ws, B_HP_SDO, std::max<uint64_t>(g->host_small[10], 1), &s_sdo));
        TRY(hipMemsetAsync(wu, 0, nU * 8, st));  // W+(u), accumulated by the fill
      }
      if (s_sdo && g->drank)
        hipLaunchKernelGGL(k_hp_dcls_fill8, dim3(gt), dim3(NT), 0, st, gv, (const uint8_t*)g->dcls, p.H, ua, nU, e0,
                           e1, (const uint32_t*)g->tile_row, (const uint64_t*)tpre, s_skeys, s_sdo,
                           (unsigned long long*)wu, (const uint8_t*)g->drank);
      else
        hipLaunchKernelGGL(k_hp_dcls_fill, dim3(gt), dim3(NT), 0, st, gv, (const uint8_t*)g->dcls, p.H, ua, nU, e0, e1,
                           (const uint32_t*)g->tile_row, (const uint64_t*)tpre, s_skeys, s_sdo,
                           (unsigned long long*)wu, (const uint8_t*)g->drank);
      TRY(hipGetLastError());
      s_sorted = true;
    } else if (p_h != ~0ull && 4 * p_h < e1 - e0) {
      // the survivor lists S(u) of the range, and W(u) with them: the row kernels walk S(u), not N(u)
      const uint64_t ns = g->dstart[p.H + 1];
      uint32_t* scnt;
      TRY(wsget(ws, B_HP_SCNT, nU, &scnt));
      TRY(wsget(ws, B_HP_SOFF, nU + 1, &s_soff));
      TRY(hipMemsetAsync(scnt, 0, nU * 4, st));
      if (ns)
        hipLaunchKernelGGL(k_hp_surv_lists<false>, dim3(grid_full(ns)), dim3(NT), 0, st, gv, (const uint32_t*)g->vbydeg,
                           ns, ua, ub, (unsigned long long*)wu, scnt, (const uint64_t*)nullptr, (uint32_t*)nullptr);
      TRY(hipGetLastError());
      TRY(scan_ws<uint32_t>(ws, B_SCAN, scnt, nU, s_soff, s_soff + nU, st));
      TRY(hipMemcpyAsync(&g->host_small[10], s_soff + nU, 8, hipMemcpyDeviceToHost, st));
      TRY(hipStreamSynchronize(st));
      TRY(wsget(ws, B_HP_SKEYS, std::max<uint64_t>(g->host_small[10], 1), &s_skeys));
      TRY(hipMemsetAsync(scnt, 0, nU * 4, st));
      if (ns)
        hipLaunchKernelGGL(k_hp_surv_lists<true>, dim3(grid_full(ns)), dim3(NT), 0, st, gv, (const uint32_t*)g->vbydeg,
                           ns, ua, ub, (unsigned long long*)wu, scnt, (const uint64_t*)s_soff, s_skeys);
      TRY(hipGetLastError());
    } else if (e1 > e0)
      hipLaunchKernelGGL(k_hp_work_edges,
                         dim3((unsigned)std::min<uint64_t>((e1 - e0 + NT * HP_WR - 1) / (NT * HP_WR) + 1, 8192)),
                         dim3(NT), 0, st, gv, p.H, ua, nU, e0, e1, (const uint32_t*)g->tile_row,
                         (unsigned long long*)wu);
  }
  uint32_t* lists[HP_NBINS];
  // bin-0 rows of a chunk by tier, then counters: [0, 6) tiers, [6, 9) work queues of bins 2, 3, 1,
  // [10] batches, [11, 14) hub pass, [16, 22) bin-1 tiers, [22, 25) their work queues; then bin-1 rows by tier
  uint32_t* tlist;
  TRY(wsget(ws, B_HP_TIER, 2 * nU + 32, &tlist));
  uint32_t* tcnt = tlist + nU;
  uint32_t* tlist1 = tlist + nU + 32;
  const int lb[HP_NBINS] = {B_HP_L0, B_HP_L1, B_HP_L2, B_HP_L3};
  for (int b = 0; b < HP_NBINS; ++b) TRY(wsget(ws, lb[b], nU, &lists[b]));
  {  // the bins' ascending row lists: count per tile, scan, scatter (hashpath.hpp k_hp_bins)
    const uint64_t nbt = (nU + HP_BTILE - 1) / HP_BTILE;
    uint32_t* bcnt;
    uint64_t* bpos;
    TRY(wsget(ws, B_HP_FLAGS, (uint64_t)HP_NBINS * nbt, &bcnt));
    TRY(wsget(ws, B_HP_BPOS, (uint64_t)HP_NBINS * nbt + 1, &bpos));
    const unsigned gb = (unsigned)std::min<uint64_t>(nbt, 8192);
    hipLaunchKernelGGL(k_hp_bins<false>, dim3(gb), dim3(NT), 0, st, (const uint64_t*)g->off, ua, nU,
                       (const uint64_t*)wu, g->hp_minbin, b1max, bcnt, (const uint64_t*)nullptr, lists[0], lists[1],
                       lists[2], lists[3], small + 24);
    TRY(hipGetLastError());
    TRY(wsget(ws, B_SCAN2, scan_scratch_words(HP_NBINS * nbt) + 16, &scan2));
    TRY(scan_ws<uint32_t>(ws, B_SCAN2, bcnt, HP_NBINS * nbt, bpos, bpos + HP_NBINS * nbt, st));
    hipLaunchKernelGGL(k_hp_bins<true>, dim3(gb), dim3(NT), 0, st, (const uint64_t*)g->off, ua, nU,
                       (const uint64_t*)wu, g->hp_minbin, b1max, bcnt, (const uint64_t*)bpos, lists[0], lists[1],
                       lists[2], lists[3], small + 24);
    TRY(hipGetLastError());
  }
  // row prefix of W(u) (wu[nU] = total)
  TRY(scan_ws<uint64_t>(ws, B_SCAN, wu, nU, pos, small + 16, st));
  TRY(hipMemcpyAsync(pos + nU, small + 16, 8, hipMemcpyDeviceToDevice, st));
  TRY(hipMemcpyAsync(&g->host_small[8], small + 16, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  const uint64_t wtot = g->host_small[8];  // >= the number of candidates
  if (wtot == 0) return NLP_OK;
  if (k > wtot) k = wtot;                   // maxEdges = all candidates
  // candidate buffer: k held + E emitted per chunk
  const uint64_t E = std::max<uint64_t>(g->hp_emit ? g->hp_emit : std::max<uint64_t>(1ull << 26, 4 * k), S);
  const uint64_t capC = k + E;
  { nlp_status s0 = cand_reserve(g, capC, 0, st); if (s0 != NLP_OK) return s0; }
  int64_t tau = -1;
  g->host_small[8] = (uint64_t)tau;
  TRY(hipMemcpyAsync(small + 8, &g->host_small[8], 8, hipMemcpyHostToDevice, st));
  uint64_t r0 = 0, q0[HP_NBINS] = {0, 0, 0, 0};
  double rate = 1.0;  // emitted candidates per unit of W(u), from the last chunk
  double real_rate = 1.0;  // the same without window padding: sizes the next chunk's emission windows
  double hub_ratio = 1.0;  // hub wedges above u per unit of W(u), from the last chunk with hub rows
  bool full = false;  // k candidates held: tau is in force
  bool retry = false; // the chunk is a retry after an emission overflow
  // the hub pass's scratch in wedges (run_hub: w, and v for AA / RA)
  const uint64_t hub_cap = std::max<uint64_t>(1, ((uint64_t)g->hp_gp * g->hp_scap * 2) / (custom ? 2 : 1));
  uint64_t target = std::min<uint64_t>(E, hub_cap);
  // Prune the held candidates: with at least k real ones (padding excluded) to
  // the canonical top k, and tau = the k-th key from then on; with fewer, only
  // the padding goes (it ranks below every real candidate: key 0, u and w
  // 0xffffffff), and no threshold is set.
  auto prune_held = [&](bool last) -> nlp_status {
    const uint64_t real = C.n - C.pad;
    uint32_t kth = 0;
    if (real >= k) {
      if (C.n > k) {
        // the last prune may fold into the 8-byte order; not for AA / RA, whose
        // top-k scores are nearly all distinct (the order would refuse them)
        nlp_status s = hp_prune(g, C, k, capC, &kth, st, last && !custom);
        if (s != NLP_OK) return s;
      }
      C.pad = 0;
      tau = (int64_t)kth;
      full = true;
      g->host_small[8] = (uint64_t)tau;
      TRY(hipMemcpyAsync(small + 8, &g->host_small[8], 8, hipMemcpyHostToDevice, st));
    } else if (C.pad) {
      nlp_status s = hp_prune(g, C, real, capC, &kth, st);
      if (s != NLP_OK) return s;
      C.pad = 0;
    }
    return NLP_OK;
  };
  while (r0 < nU) {
    hipLaunchKernelGGL(k_hp_bounds, dim3(1), dim3(64), 0, st, (const uint64_t*)pos, nU, r0, target, ua,
                       (const uint32_t*)lists[0], (const uint32_t*)lists[1], (const uint32_t*)lists[2],
                       (const uint32_t*)lists[3], (const uint64_t*)(small + 24), small + 16);
    TRY(hipGetLastError());
    TRY(hipMemsetAsync(small, 0, 8 * HPC_NCTR, st));
    // bounds are read back with the counters below; the kernels read them from the host copy
    TRY(hipMemcpyAsync(&g->host_small[16], small + 16, 40, hipMemcpyDeviceToHost, st));
    TRY(hipMemcpyAsync(&g->host_small[40], pos + r0, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    const uint64_t r1 = g->host_small[16];
    uint64_t q1[HP_NBINS];
    for (int b = 0; b < HP_NBINS; ++b) q1[b] = g->host_small[17 + b];
    TRY(hipMemcpyAsync(&g->host_small[41], pos + r1, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    const uint64_t wchunk = g->host_small[41] - g->host_small[40];
    HpArgs a{};
    a.g = gv;
    a.ctn = g->maxdeg + 1;
    a.S = S;
    a.H = p.H;
    a.metric = p.metric;
    a.min_score = p.min_score;
    a.ckey = (uint32_t*)ws.p[B_CKEY];
    a.cu = (uint32_t*)ws.p[B_CU];
    a.cw = (uint32_t*)ws.p[B_CW];
    a.cs = (float*)ws.p[B_CS];
    a.base = C.n;
    a.cap = capC - C.n;
    a.tau = (const int64_t*)(small + 8);
    a.ctr = (unsigned long long*)small;
    a.soff = s_skeys ? s_soff : nullptr;
    a.scn = s_skeys ? s_scn : nullptr;
    a.skeys = s_skeys;
    a.ssorted = s_sorted ? 1 : 0;
    a.kdeg = g->kdeg;
    a.sdo = s_sdo;
    a.sua = ua;
    a.xs = g->xs;
    a.win = 0;
    a.uxf = g->hp_uxf;
    // phase ticks (k_hp_batch, k_hh_accum's sort mode; diagnostic: small[56, 60) with NLP_TRACE_HUB=1)
    static const bool trace_hub = getenv("NLP_TRACE_HUB") && getenv("NLP_TRACE_HUB")[0] == '1';
    a.ph = nullptr;  // run_hub points its copy at small[56, 60) when tracing
    if (trace_hub) TRY(hipMemsetAsync(small + 56, 0, 48, st));
    // NLP_TRACE_BATCH=1 (diagnostic): k_hp_batch's wave time per phase into small[64, 68)
    static const bool trace_batch = getenv("NLP_TRACE_BATCH") && getenv("NLP_TRACE_BATCH")[0] == '1';
    if (trace_batch) TRY(hipMemsetAsync(small + 64, 0, 32, st));
    const uint64_t n0 = q1[0] - q0[0], n1 = q1[1] - q0[1];
    bool batch_timed = false;
    if (n0) {
      // bin 0 by table-size tier (hashpath.hpp:k_hp_tier): counts, scatter, one launch per tier
      TRY(hipMemsetAsync(tcnt, 0, 8 * sizeof(uint32_t), st));
      const unsigned gt = (unsigned)std::min<uint64_t>((n0 + NT - 1) / NT, 512);
      hipLaunchKernelGGL(k_hp_tier<false>, dim3(gt), dim3(NT), 0, st, (const uint32_t*)(lists[0] + q0[0]), n0,
                         (const uint64_t*)wu, ua, tcnt, tlist);
      hipLaunchKernelGGL(k_hp_tier<true>, dim3(gt), dim3(NT), 0, st, (const uint32_t*)(lists[0] + q0[0]), n0,
                         (const uint64_t*)wu, ua, tcnt, tlist);
      TRY(hipGetLastError());
      const unsigned gr = (unsigned)std::min<uint64_t>((n0 + NWAVE - 1) / NWAVE, 8192);
      const uint32_t* tl = tlist;
      const uint32_t* tc = tcnt;
      const int wbits = bits_for(S - 1);
      if (g->hp_batch && s_skeys && wbits <= 26) {
        // tiers 0 and 1 in row batches (hashpath.hpp:k_hp_batch), tier 2 a wave per row
        uint64_t *bw, *bpre;
        uint32_t* bst;
        TRY(wsget(ws, B_HB_W, n0, &bw));
        TRY(wsget(ws, B_HB_PRE, n0 + 1, &bpre));
        TRY(wsget(ws, B_HB_START, (wchunk + HB_ROWCOST * n0) / 256 + 8, &bst));
        uint32_t* nbat = tcnt + 10;
        const uint64_t bwid = 256;  // tiers 0 and 1 (W <= 256) together, 1024-entry tables
        LAUNCH(k_hp_batch_w, n0, st, (const uint32_t*)tl, n0, tc, 0, 1, (const uint64_t*)wu, ua, bw);
        TRY(scan_ws<uint64_t>(ws, B_SCAN, bw, n0, bpre, bpre + n0, st));
        TRY(hipMemsetAsync(nbat, 0, 4, st));
        LAUNCH(k_hp_batch_starts, n0, st, (const uint64_t*)bpre, tc, 0, 1, bwid, bst, nbat);
        TRY(hipGetLastError());
        unsigned gb = gr;  // row batches
        if (!retry) {
          // persistent waves (one resident round) reserving emission windows: about an
          // eighth of a wave's share of the chunk's wedge bound per window, so the
          // padding stays below an eighth of the chunk's emission bound; a chunk too
          // small for a window of HP_STG per wave, or the retry of an overflowed
          // chunk, reserves per flush
          const unsigned grb = std::min<unsigned>(gr, g->occ_hb);
          // from the last chunk's REAL emissions: with a threshold in force a chunk emits a few percent
          // of its wedges, and windows sized by the wedge bound padded ~1.3e7 slots per chunk of the
          // C5 IHub shards (every chunk then filled the buffer and forced a prune)
          const uint64_t per = (uint64_t)(real_rate * (double)wchunk) / ((uint64_t)grb * NWAVE * 8 + 1);
          if (per >= (uint64_t)HP_STG) {
            a.win = (uint32_t)std::min<uint64_t>(HP_WIN, per);
            gb = grb;
          }
        }
        TRY(hipEventRecord(g->ev[5], st));  // the dominant kernel of path 4, timed on its own stream
        HpArgs ab = a;
        ab.ph = trace_batch ? (unsigned long long*)(small + 64) : nullptr;
        if (custom) hipLaunchKernelGGL((k_hp_batch<true, 1024, 128>), dim3(gb), dim3(NT), 0, st, ab, tl, tc, 0, 1, (const uint32_t*)bst, (const uint32_t*)nbat, (const uint64_t*)wu, ua, wbits);
        else if (a.kdeg) hipLaunchKernelGGL((k_hp_batch<false, 1024, 128, true>), dim3(gb), dim3(NT), 0, st, ab, tl, tc, 0, 1, (const uint32_t*)bst, (const uint32_t*)nbat, (const uint64_t*)wu, ua, wbits);
        else hipLaunchKernelGGL((k_hp_batch<false, 1024, 128>), dim3(gb), dim3(NT), 0, st, ab, tl, tc, 0, 1, (const uint32_t*)bst, (const uint32_t*)nbat, (const uint64_t*)wu, ua, wbits);
        TRY(hipGetLastError());
        TRY(hipEventRecord(g->ev[6], st));
        batch_timed = true;
        a.win = 0;  // the other row kernels reserve per flush
        if (custom) hipLaunchKernelGGL((k_hp_wave<true>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 2);
        else if (a.kdeg) hipLaunchKernelGGL((k_hp_wave<false, HP_WT, HP_STG, true>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 2);
        else hipLaunchKernelGGL((k_hp_wave<false>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 2);
      } else if (custom) {
        hipLaunchKernelGGL((k_hp_wave<true, 256, 256>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 0);
        hipLaunchKernelGGL((k_hp_wave<true, 512, 256>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 1);
        hipLaunchKernelGGL((k_hp_wave<true>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 2);
      } else {
        hipLaunchKernelGGL((k_hp_wave<false, 256, 256>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 0);
        hipLaunchKernelGGL((k_hp_wave<false, 512, 256>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 1);
        hipLaunchKernelGGL((k_hp_wave<false>), dim3(gr), dim3(NT), 0, st, a, tl, n0, wu, ua, tc, 2);
      }
      TRY(hipGetLastError());
    }
    TRY(hipMemsetAsync(tcnt + 6, 0, 3 * sizeof(uint32_t), st));  // work queues of bins 2, 3 and 1
    bool b1_done = false;
    if (n1 && g->hp_hub && g->hp_hub_min == 1) {
      nlp_status sh = run_hub(g, a, lists[1] + q0[1], n1, nullptr, 0, wu, ua, custom, scan, tcnt + 11, &b1_done, st);
      if (sh != NLP_OK) return sh;
    }
    if (n1 && !b1_done && custom && a.sdo && a.ssorted && g->hp_rowb) {
      // AA / RA: bin 1 (W+ <= 2048) by table tier (k_hp_rowo), ordered tables over 256 threads
      TRY(hipMemsetAsync(tcnt + 16, 0, 9 * sizeof(uint32_t), st));
      const unsigned gt = (unsigned)std::min<uint64_t>((n1 + NT - 1) / NT, 512);
      const uint64_t rt0 = g->hp_rowb >= 2 ? 0 : HP_RTIER0, rt1 = HP_RTIER1;
      hipLaunchKernelGGL(k_hp_tier<false>, dim3(gt), dim3(NT), 0, st, (const uint32_t*)(lists[1] + q0[1]), n1,
                         (const uint64_t*)wu, ua, tcnt + 16, tlist1, rt0, rt1);
      hipLaunchKernelGGL(k_hp_tier<true>, dim3(gt), dim3(NT), 0, st, (const uint32_t*)(lists[1] + q0[1]), n1,
                         (const uint64_t*)wu, ua, tcnt + 16, tlist1, rt0, rt1);
      TRY(hipGetLastError());
      const unsigned grw = (unsigned)std::min<uint64_t>(n1, 4096);
      hipLaunchKernelGGL((k_hp_rowo<2048>), dim3(grw), dim3(HP_RNT), 0, st, a, (const uint32_t*)tlist1, (const uint32_t*)(tcnt + 16), 0, wu, ua, tcnt + 22);
      hipLaunchKernelGGL((k_hp_rowo<4096>), dim3(grw), dim3(HP_RNT), 0, st, a, (const uint32_t*)tlist1, (const uint32_t*)(tcnt + 16), 1, wu, ua, tcnt + 23);
      TRY(hipGetLastError());
      b1_done = true;
    }
    if (n1 && !b1_done && !custom && a.kdeg && g->hp_rowb) {
      // count metrics: bin 1 by table tier (k_hp_rowb), 256-thread workgroups
      TRY(hipMemsetAsync(tcnt + 16, 0, 9 * sizeof(uint32_t), st));
      const unsigned gt = (unsigned)std::min<uint64_t>((n1 + NT - 1) / NT, 512);
      const uint64_t rt0 = g->hp_rowb >= 2 ? 0 : HP_RTIER0, rt1 = g->hp_rowb == 2 ? 0 : HP_RTIER1;
      hipLaunchKernelGGL(k_hp_tier<false>, dim3(gt), dim3(NT), 0, st, (const uint32_t*)(lists[1] + q0[1]), n1,
                         (const uint64_t*)wu, ua, tcnt + 16, tlist1, rt0, rt1);
      hipLaunchKernelGGL(k_hp_tier<true>, dim3(gt), dim3(NT), 0, st, (const uint32_t*)(lists[1] + q0[1]), n1,
                         (const uint64_t*)wu, ua, tcnt + 16, tlist1, rt0, rt1);
      TRY(hipGetLastError());
      // one launch per tier (its rows and count read on the device, no host wait)
      const unsigned grw = (unsigned)std::min<uint64_t>(n1, 4096);
      // (128-thread workgroups for the 2048-entry tier measured no faster: 4.38 vs 4.13 ms on C4 JAC H=16)
      hipLaunchKernelGGL((k_hp_rowb<2048>), dim3(grw), dim3(HP_RNT), 0, st, a, (const uint32_t*)tlist1, (const uint32_t*)(tcnt + 16), 0, wu, ua, tcnt + 22);
      hipLaunchKernelGGL((k_hp_rowb<4096>), dim3(grw), dim3(HP_RNT), 0, st, a, (const uint32_t*)tlist1, (const uint32_t*)(tcnt + 16), 1, wu, ua, tcnt + 23);
      hipLaunchKernelGGL((k_hp_rowb<8192>), dim3(grw), dim3(HP_RNT), 0, st, a, (const uint32_t*)tlist1, (const uint32_t*)(tcnt + 16), 2, wu, ua, tcnt + 24);
      TRY(hipGetLastError());
      b1_done = true;
    }
    if (n1 && !b1_done) {
      const unsigned gr = (unsigned)std::min<uint64_t>(n1, 2048);
      if (custom) hipLaunchKernelGGL((k_hp_block<true, false>), dim3(gr), dim3(HP_BNT), 0, st, a, lists[1] + q0[1], n1, wu, ua, (uint32_t*)nullptr, 13, tcnt + 8);
      else if (a.kdeg) hipLaunchKernelGGL((k_hp_block<false, false, true>), dim3(gr), dim3(HP_BNT), 0, st, a, lists[1] + q0[1], n1, wu, ua, (uint32_t*)nullptr, 13, tcnt + 8);
      else hipLaunchKernelGGL((k_hp_block<false, false>), dim3(gr), dim3(HP_BNT), 0, st, a, lists[1] + q0[1], n1, wu, ua, (uint32_t*)nullptr, 13, tcnt + 8);
      TRY(hipGetLastError());
    }
    bool hub_done = false;
    uint64_t hub_w = 0;  // the chunk's hub wedges above u (run_hub's count pass)
    if (g->hp_hub && (q1[2] - q0[2]) + (q1[3] - q0[3]) > 0) {
      nlp_status sh = run_hub(g, a, lists[2] + q0[2], q1[2] - q0[2], lists[3] + q0[3], q1[3] - q0[3], wu, ua, custom,
                              scan, tcnt + 11, &hub_done, st, &hub_w);  // tcnt[11, 14): queue, item and heavy counts
      if (sh != NLP_OK) return sh;
    }
    for (int b = 2; b < HP_NBINS && !hub_done; ++b) {  // rows beyond an LDS table: w-bucket partitioning
      const uint64_t nb = q1[b] - q0[b];
      if (!nb) continue;
      // fewer rows than workgroups: slice each row's w-buckets over several workgroups
      const uint32_t nsl = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(g->hp_gp / nb, 256));
      const unsigned gr = (unsigned)std::min<uint64_t>(nb * nsl, g->hp_gp);
      if (custom) hipLaunchKernelGGL(k_hp_part<true>, dim3(gr), dim3(HP_BNT), 0, st, a, lists[b] + q0[b], nb, wu, ua, g->hp_scratch, g->hp_scap, nsl, tcnt + 4 + b);
      else hipLaunchKernelGGL(k_hp_part<false>, dim3(gr), dim3(HP_BNT), 0, st, a, lists[b] + q0[b], nb, wu, ua, g->hp_scratch, g->hp_scap, nsl, tcnt + 4 + b);
      TRY(hipGetLastError());
    }
    TRY(hipMemcpyAsync(g->host_small, small, 8 * HPC_NCTR, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    const uint64_t emitted = g->host_small[HPC_EMIT];
    if (trace_batch) {
      uint64_t pb[4] = {0, 0, 0, 0};
      TRY(hipMemcpy(pb, small + 64, 32, hipMemcpyDeviceToHost));
      const double tot = (double)(pb[0] + pb[1] + pb[2] + pb[3]) + 1e-9;
      fprintf(stderr, "nlp batch: chunk %u wave ticks (10 ns) setup %llu (%.1f%%) wedges %llu (%.1f%%) exclusion %llu "
              "(%.1f%%) drain %llu (%.1f%%)\n", *nchunks, (unsigned long long)pb[0], 100.0 * pb[0] / tot,
              (unsigned long long)pb[1], 100.0 * pb[1] / tot, (unsigned long long)pb[2], 100.0 * pb[2] / tot,
              (unsigned long long)pb[3], 100.0 * pb[3] / tot);
    }
    {
      static const bool trace = getenv("NLP_TRACE_HUB") && getenv("NLP_TRACE_HUB")[0] == '1';
      if (trace) {
        uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
        TRY(hipMemcpy(ph, small + 56, 48, hipMemcpyDeviceToHost));
        fprintf(stderr, "nlp hub: chunk %u rows %llu wedges %llu hub wedges %llu of which in HH_BIG items %llu; "
                "ticks (10 ns, summed over workgroups): sort mode load %llu sort %llu exclusion %llu runs %llu; "
                "hash items %llu, the longest %llu\n",
                *nchunks, (unsigned long long)(r1 - r0), (unsigned long long)g->host_small[HPC_WEDGE],
                (unsigned long long)hub_w, (unsigned long long)g->host_small[HPC_BIGW], (unsigned long long)ph[0],
                (unsigned long long)ph[1], (unsigned long long)ph[2], (unsigned long long)ph[3],
                (unsigned long long)ph[4], (unsigned long long)ph[5]);
      }
    }
    if (batch_timed) {
      float ms = 0;
      TRY(hipEventElapsedTime(&ms, g->ev[5], g->ev[6]));
      C.hot_ms += ms;
      C.hot_bytes += g->host_small[HPC_HOTB];
      ++C.hot_launches;
    }
    if (g->host_small[HPC_ERR]) return NLP_ERR_DEVICE;
    if (emitted > a.cap) {
      // overflow: nothing of this chunk is kept; prune what is held and retry a smaller chunk
      // (without emission windows: their padding must not keep a retry overflowing)
      retry = true;
      rate = std::max(rate, (double)emitted / (double)std::max<uint64_t>(wchunk, 1));
      target = std::max<uint64_t>(1, wchunk / 4);
      if (C.n > k || C.pad) {
        nlp_status s = prune_held(false);
        if (s != NLP_OK) return s;
      } else if (r1 == r0 + 1) {
        return NLP_ERR_DEVICE;  // one row cannot exceed E >= S free slots
      }
      continue;
    }
    ++*nchunks;
    retry = false;
    // row bookkeeping (W+(u), survivor prefix, bins, tiers: ~64 B per row), per wedge its key and
    // entry degree plus its packed survivor entry at most (16 B of the chunk's bound), 16 B per emission
    C.call_bytes += 64 * (r1 - r0) + 16 * wchunk + 16 * emitted;
    C.pad += g->host_small[HPC_PAD];
    C.n += emitted;
    C.total += g->host_small[HPC_CAND];
    C.nan += g->host_small[HPC_NAN];
    C.wedges += g->host_small[HPC_WEDGE];
    rate = (double)emitted / (double)std::max<uint64_t>(wchunk, 1);
    real_rate = (double)(emitted - std::min<uint64_t>(emitted, g->host_small[HPC_PAD])) /
                (double)std::max<uint64_t>(wchunk, 1);
    // the hub rows' real wedges (above u) per unit of the chunk's bound W(u) (every w): the next
    // chunk's bound may be that much larger for the same hub scratch (IHub rows of high ids
    // enumerate a small part of their lists)
    if (hub_w > 0 && wchunk > 0) hub_ratio = std::min(1.0, (double)hub_w / (double)wchunk);
    r0 = r1;
    for (int b = 0; b < HP_NBINS; ++b) q0[b] = q1[b];
    if ((C.n > k && C.n > k + E / 2) || (r0 >= nU && (C.n > k || C.pad))) {
      nlp_status s = prune_held(r0 >= nU);
      if (s != NLP_OK) return s;
    }
    // next chunk: aim at half of the free buffer at the last emission rate, and
    // at most the hub pass's scratch in wedges: a chunk beyond it would run its
    // hub rows through k_hp_part (with a threshold in force the emission rate
    // is tiny and the emission bound alone grew IHub chunks to 3e11 wedges:
    // the C5 shard 0 ran at 5.8e9 instead of 2.4e10 wedges/s)
    const uint64_t free_slots = capC - C.n;
    const double want = 0.5 * (double)free_slots / std::max(rate, 1e-9);
    target = (uint64_t)std::min(want, 1e18);
    if (!full && target > free_slots) target = free_slots;  // no threshold yet: emissions <= W(u)
    target = std::min<uint64_t>(target, (uint64_t)std::min(1e18, 0.8 * (double)hub_cap / std::max(hub_ratio, 0.02)));
    if (target == 0) target = 1;
  }
  // held candidates are unordered: the caller orders them (hp_final_order)
  return NLP_OK;
}

// ================================================================ fast path
// Path 1 + selection + ordering with no host synchronisation: every kernel
// reads its sizes from device counters and buffers are sized by the wedge
// capacity.  prepare_fast allocates (never inside a capture); launch_fast only
// launches, so it can be captured into a hipGraph and replayed.
struct FastBufs {
  uint32_t *ucnt, *cursor;
  uint64_t* uoff;
  StageBufs sb;
  BigItem* big;
  uint32_t *ck, *cu, *cw, *tk, *tu, *tw, *k0, *k1, *v0, *v1;
  float *cs, *ts;
  uint64_t *aggs, *arena;
  uint64_t aU, aW, ntW, arena_words;
};

uint64_t ws_fingerprint(const Workspace& ws) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < NBUF; ++i) {
    h = (h ^ (uint64_t)(uintptr_t)ws.p[i]) * 1099511628211ull;
    h = (h ^ (uint64_t)ws.bytes[i]) * 1099511628211ull;
  }
  return h;
}

nlp_status prepare_fast(nlp_graph* g, const Params& p, FastBufs& f, hipStream_t st) {
  const uint64_t S = g->span;
  const uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S), nU = ub - ua;
  Workspace& ws = g->ws;
  if (ws.bytes[B_UCNT] < S * 4 || ws.bytes[B_IEP] < S * 4) {
    uint32_t *a, *b;
    TRY(wsget(ws, B_UCNT, S, &a));
    TRY(wsget(ws, B_IEP, S, &b));
    TRY(hipMemsetAsync(a, 0, S * 4, st));
    TRY(hipMemsetAsync(b, 0, S * 4, st));
  }
  f.ucnt = (uint32_t*)ws.p[B_UCNT];
  f.cursor = (uint32_t*)ws.p[B_IEP];
  const uint64_t capW = g->capW;
  TRY(wsget(ws, B_UOFF, S, &f.uoff));
  nlp_status s = stage_bufs(g, capW, 0, f.sb);
  if (s != NLP_OK) return s;
  TRY(wsget(ws, B_BIG, std::max<uint64_t>(nU, 1), &f.big));
  s = cand_reserve(g, capW, 0, st);
  if (s != NLP_OK) return s;
  f.ck = (uint32_t*)ws.p[B_CKEY]; f.cu = (uint32_t*)ws.p[B_CU]; f.cw = (uint32_t*)ws.p[B_CW]; f.cs = (float*)ws.p[B_CS];
  TRY(wsget(ws, B_TKEY, capW, &f.tk));
  TRY(wsget(ws, B_TU, capW, &f.tu));
  TRY(wsget(ws, B_TW, capW, &f.tw));
  TRY(wsget(ws, B_TS, capW, &f.ts));
  TRY(wsget(ws, B_OK0, capW, &f.k0));
  TRY(wsget(ws, B_OK1, capW, &f.k1));
  TRY(wsget(ws, B_OV0, capW, &f.v0));
  TRY(wsget(ws, B_OV1, capW, &f.v1));
  constexpr int IPT_S = 16, IPT_W = 4;
  f.aU = (nU + NT * IPT_S - 1) / (NT * IPT_S) + 1;
  f.aW = (capW + NT * IPT_W - 1) / (NT * IPT_W) + 1;
  TRY(wsget(ws, B_FAGG, f.aU + 2 * f.aW, &f.aggs));
  f.ntW = (capW + OS_TILE - 1) / OS_TILE + 1;
  f.arena_words = AR_DESC + 4 * f.ntW * RS_BINS;
  TRY(wsget(ws, B_FARENA, f.arena_words, &f.arena));
  return NLP_OK;
}

// seg < 0 launches everything and records the timing events; seg = 0..3
// launches one segment only (the hipGraph pieces; events go between them).
nlp_status launch_fast(nlp_graph* g, const Params& p, const FastBufs& f, EdgeOut* d_out, hipStream_t st, int seg) {
  const uint64_t S = g->span;
  const uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S), nU = ub - ua;
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  const GraphView gv = view_of(g, p.metric, p.maxf2);
  const uint64_t capW = g->capW;
  constexpr int IPT_S = 16, IPT_W = 4;
  uint64_t *gU = f.aggs, *gW = f.aggs + f.aU, *gT = gW + f.aW;
  uint64_t* ctr = f.arena;
  uint64_t* sel = f.arena + AR_SEL;
  uint32_t* tickets = (uint32_t*)(f.arena + AR_TICKETS);
  uint32_t* selhist = (uint32_t*)(f.arena + AR_SELHIST);
  uint32_t* oshist = (uint32_t*)(f.arena + AR_OSHIST);
  uint64_t* desc = f.arena + AR_DESC;
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  const StageBufs& sb = f.sb;
  CtrInit ci;
  for (int i = 0; i < NCTR; ++i) ci.v[i] = 0;
  ci.v[C_N_URANGE] = nU;
  ci.v[10] = S;
  BucketsP1 bk{f.uoff, f.ucnt};
  const unsigned gtiles = (unsigned)std::min<uint64_t>(std::max<uint64_t>((nU + GT_TILE - 1) / GT_TILE, 1), 65535);
  if (seg < 0) TRY(hipEventRecord(g->ev[0], st));
  if (seg < 0 || seg == 0) {
    hipLaunchKernelGGL(k_arena_init, dim3(std::min<uint64_t>(1024, (f.arena_words + NT - 1) / NT)), dim3(NT), 0, st,
                       f.arena, f.arena_words, ci);
    // ---- candidates (path 1)
    hipLaunchKernelGGL(k_p1_pass<false>, dim3(p1_grid(S)), dim3(NT), 0, st, gv, S, p.H, ua, ub, f.ucnt,
                       (const uint64_t*)nullptr, capW, sb.bucket, ctr);
    TRY(hipGetLastError());
    TRY((rts_scan<F_UOff, IPT_S>(F_UOff{f.ucnt, f.uoff, ua}, &ctr[C_N_URANGE], nU, gU, &ctr[C_W], st)));
    hipLaunchKernelGGL(k_p1_pass<true>, dim3(p1_grid(S)), dim3(NT), 0, st, gv, S, p.H, ua, ub, f.cursor,
                       (const uint64_t*)f.uoff, capW, sb.bucket, ctr);
    TRY(hipGetLastError());
  }
  if (seg < 0) TRY(hipEventRecord(g->ev[3], st));
  if (seg < 0 || seg == 1) {
    if (custom)
      hipLaunchKernelGGL((k_group_tiles<BucketsP1, true>), dim3(gtiles), dim3(NT), 0, st, gv, bk, ua, ub, p.metric,
                         p.min_score, sb.bucket, capW, sb.st, f.big, ctr, f.ucnt, f.cursor);
    else
      hipLaunchKernelGGL((k_group_tiles<BucketsP1, false>), dim3(gtiles), dim3(NT), 0, st, gv, bk, ua, ub, p.metric,
                         p.min_score, sb.bucket, capW, sb.st, f.big, ctr, f.ucnt, f.cursor);
    TRY(hipGetLastError());
  }
  if (seg < 0) TRY(hipEventRecord(g->ev[4], st));
  if (seg < 0 || seg == 2) {
    if (custom) {
      hipLaunchKernelGGL((k_group_big<true>), dim3(256), dim3(NT), 0, st, gv, p.metric, p.min_score, sb.bucket, sb.st,
                         (const BigItem*)f.big, ctr);
      LAUNCH_FULL(k_score_runs<true>, capW, st, gv, p.metric, p.min_score, ctr, capW, sb.st);
    } else {
      hipLaunchKernelGGL((k_group_big<false>), dim3(256), dim3(NT), 0, st, gv, p.metric, p.min_score, sb.bucket, sb.st,
                         (const BigItem*)f.big, ctr);
      LAUNCH_FULL(k_score_runs<false>, capW, st, gv, p.metric, p.min_score, ctr, capW, sb.st);
  }
  TRY(hipGetLastError());
  hipLaunchKernelGGL(k_clamp_n, dim3(1), dim3(64), 0, st, ctr, (uint64_t)C_W, capW, (uint64_t)11);
  TRY((rts_scan<F_Compact, IPT_W>(F_Compact{sb.st, f.ck, f.cu, f.cw, f.cs, ctr, &ctr[C_NAN]}, &ctr[11], capW, gW,
                                  &ctr[C_C], st)));
  }
  if (seg < 0) TRY(hipEventRecord(g->ev[1], st));
  if (seg < 0 || seg == 3) {
    // ---- top-k selection (only when candidates > max_edges; kernels no-op otherwise)
    hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(64), 0, st, ctr, sel, p.max_edges);
    for (int pass = 0; pass < 3; ++pass) {
      LAUNCH(k_sel_hist, capW, st, (const uint32_t*)f.ck, &ctr[C_SEL_N], pass, (const uint64_t*)sel, selhist);
      hipLaunchKernelGGL(k_sel_pick2, dim3(1), dim3(NT), 0, st, selhist, pass, sel, (const uint64_t*)ctr);
  }
  TRY(hipGetLastError());
  TRY((rts_scan<F_Sel, IPT_W>(F_Sel{f.ck, f.cu, f.cw, f.cs, sel, f.tk, f.tu, f.tw, f.ts}, &ctr[C_SEL_N], capW, gT,
                              nullptr, st)));
  // ---- canonical order: stable sort by score key descending
  CandBufs ca{f.ck, f.cu, f.cw, f.cs}, cb{f.tk, f.tu, f.tw, f.ts};
  LAUNCH(k_desc_keys_sel, capW, st, ca, cb, (const uint64_t*)ctr, f.k0, f.v0);
  hipLaunchKernelGGL(k_os_hist, dim3(64), dim3(NT), 0, st, (const uint32_t*)f.k0, (const uint64_t*)&ctr[C_OUT_N],
                     oshist);
  TRY(hipGetLastError());
  uint32_t *ka = f.k0, *va = f.v0, *kb = f.k1, *vb = f.v1;
  for (int pass = 0; pass < 4; ++pass) {
    hipLaunchKernelGGL(k_os_pass, dim3((unsigned)f.ntW), dim3(NT), 0, st, ka, va, kb, vb,
                       (const uint64_t*)&ctr[C_OUT_N], 8 * pass, oshist + pass * RS_BINS, tickets + pass,
                       desc + (uint64_t)pass * f.ntW * RS_BINS, err);
    TRY(hipGetLastError());
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  LAUNCH(k_gather_sel, capW, st, (const uint32_t*)va, ca, cb, (const uint64_t*)ctr, d_out);
  TRY(hipGetLastError());
  TRY(hipMemcpyAsync(g->host_small, ctr, NCTR * 8, hipMemcpyDeviceToHost, st));
  }
  if (seg < 0) TRY(hipEventRecord(g->ev[2], st));
  return NLP_OK;
}

// ---------------------------------------------------------------- sort-grouped fast path
struct SpBufs {
  uint32_t* surv;
  uint64_t *rk0, *rk1;
  uint32_t *rv0, *rv1, *cu, *cw, *ok0, *ok1, *ov0, *ov1;
  float *stash, *cs;
  uint32_t* segcnt;  // k_sp_runs: candidates per RU_SEG-record segment (gapped layout)
  uint64_t* arena;
  uint64_t arena_words;
  uint64_t d_surv, d_exp, d_run, d_rec, d_ord;  // descriptor offsets in the arena (u64 words)
  uint64_t d_cm;                                // counted passes: 4 count matrices of CP_MAXT x 256 u32 (after d_ord)
  uint64_t d_tick;                              // SP_NTICK u32 ticket counters (one per ticketed launch)
  uint64_t d_wsum;                              // WSUM_COPIES wedge-count copies (direct emission)
  uint64_t d_bcur;                              // DX_MAXB x EXB_SUB u32 bucket cursors (direct emission)
  uint64_t d_ts;                                // TS_WORDS u64 call-timing stamps (sortpath.hpp ts_enter)
  bool direct;    // count metrics, one MSD pass: k_sp_excount + k_sp_exemit + k_sp_group instead of
                  // k_sp_expand + MSD pass + k_sp_bucket
  int dbits, dshift;  // direct buckets: the key's top dbits bits (key >> dshift)
  bool fused;         // direct, small W: fixed-capacity buckets (k_sp_exbucket) sorted and scored by
                      // k_sp_grouprun, one workgroup per bucket
  int caplog;         // fused: log2 of the slots per bucket
  uint64_t* bkt;      // fused: the buckets' record slots (2^(dbits + caplog) keys)
  ArenaZero zero;     // arena words reset per call (fused: counters, score-digit histograms, descriptors up to the
                      // survivor tiles; its ordering descriptors clean themselves)
  uint64_t ostride;                             // u32 onesweep descriptors per pass
  uint64_t ostride11;                           // the same for 11-bit digits (the fused path's three passes)
  bool ord11;                                   // fused path: three 11-bit passes
  bool small;                                   // fused path: k_sp_order_rank orders all candidates (one launch)
  bool counted;                                 // fused path: passes 2-4 are k_sp_cpass (tile digit counts from the
                                                // pass before, count matrix p at d_cm; the last pass gathers)
  int wbits, passes;
  bool msd;       // one MSD pass on the top 8 key bits + k_sp_bucket (else: full LSD sort + k_sp_scan<F_Runs>)
  int msd_shift;  // shift of the lowest MSD digit (the fine-bucket boundary in split mode)
  int msd_passes; // MSD passes before the group sort (split mode: 1 or 2; fused bucket kernel: 1)
  bool split;     // msd: k_sp_bucket sorts only, k_sp_runs scores (else k_sp_bucket does both)
  bool dindex;    // survivors = a prefix of the degree-class index (no k_sp_survivors)
  uint64_t nv;    // survivors when dindex
  const uint32_t* survivors;
};

inline int key_bits(uint64_t x) {  // bits needed for the values 0..x (at least 1)
  int b = 1;
  while (b < 64 && (x >> b)) ++b;
  return b;
}

// Degree-class index of classes 1..H restricted to the intermediates with an
// in-neighbour in [ua, ub) (k_range_index), built on the graph's stream once per
// (range, H) and kept; every ranged call checks it before its kernels run, so a
// replayed graph of another range never sees a stale index.
nlp_status ensure_range_index(nlp_graph* g, uint64_t ua, uint64_t ub, uint32_t H) {
  if (g->rx_H >= H && g->rx_ua == ua && g->rx_ub == ub) return NLP_OK;
  hipStream_t st = g->stream;
  if (!g->rx_vbydeg) {
    TRY(hipMalloc(&g->rx_vbydeg, std::max<uint64_t>(g->dstart[DCAP + 1], 1) * 4));
    TRY(hipMalloc(&g->rx_cnt, (DCAP + 1) * 8));
  }
  const uint64_t n = g->dstart[H + 1];
  const GraphView gv = view_of(g, M_CN);
  TRY(hipMemsetAsync(g->rx_cnt, 0, (DCAP + 1) * 8, st));
  hipLaunchKernelGGL(k_range_index<false>, dim3(grid_for(n)), dim3(NT), 0, st, gv, (const uint32_t*)g->vbydeg, n, H,
                     ua, ub, g->rx_cnt, (uint32_t*)nullptr);
  TRY(hipGetLastError());
  std::vector<unsigned long long> c(H + 1);
  TRY(hipMemcpyAsync(c.data(), g->rx_cnt, (H + 1) * 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  g->rx_dstart.assign(H + 2, 0);
  for (uint32_t d = 1; d <= H; ++d) g->rx_dstart[d + 1] = g->rx_dstart[d] + c[d];
  std::vector<unsigned long long> cur(g->rx_dstart.begin(), g->rx_dstart.begin() + H + 1);
  TRY(hipMemcpyAsync(g->rx_cnt, cur.data(), (H + 1) * 8, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_range_index<true>, dim3(grid_for(n)), dim3(NT), 0, st, gv, (const uint32_t*)g->vbydeg, n, H, ua,
                     ub, g->rx_cnt, g->rx_vbydeg);
  TRY(hipGetLastError());
  TRY(hipStreamSynchronize(st));
  g->rx_ua = ua;
  g->rx_ub = ub;
  g->rx_H = H;
  return NLP_OK;
}

nlp_status prepare_sp(nlp_graph* g, const Params& p, SpBufs& f, bool msd, int msd_passes) {
  const uint64_t S = g->span;
  const uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S);
  const uint64_t capW = g->capW;
  Workspace& ws = g->ws;
  TRY(wsget(ws, B_SP_SURV, S, &f.surv));
  TRY(wsget(ws, B_SP_RK0, capW, &f.rk0));
  TRY(wsget(ws, B_SP_RK1, capW, &f.rk1));
  TRY(wsget(ws, B_SP_RV0, capW, &f.rv0));
  TRY(wsget(ws, B_SP_RV1, capW, &f.rv1));
  TRY(wsget(ws, B_SP_STASH, capW, &f.stash));
  TRY(wsget(ws, B_SP_CU, capW, &f.cu));
  TRY(wsget(ws, B_SP_CW, capW, &f.cw));
  TRY(wsget(ws, B_SP_CS, capW, &f.cs));
  TRY(wsget(ws, B_SP_OK0, capW, &f.ok0));
  TRY(wsget(ws, B_SP_OK1, capW, &f.ok1));
  TRY(wsget(ws, B_SP_OV0, capW, &f.ov0));
  TRY(wsget(ws, B_SP_OV1, capW, &f.ov1));
  TRY(wsget(ws, B_SP_SEGCNT, (capW + RU_SEG - 1) / RU_SEG + 1, &f.segcnt));
  f.wbits = key_bits(S ? S - 1 : 0);
  const int ubits = key_bits(ub > ua ? ub - ua - 1 : 0);
  f.passes = (f.wbits + ubits + 7) / 8;
  f.msd = msd;
  f.split = msd && g->split_bucket;
  f.msd_passes = f.split ? std::min(msd_passes, std::max(1, (f.wbits + ubits) / 8)) : 1;
  f.msd_shift = std::max(0, f.wbits + ubits - 8 * f.msd_passes);
  f.direct = g->direct_emit && f.split && f.msd_passes == 1 && g->group_sort != 1 && p.metric != M_AA &&
             p.metric != M_RA;
  {  // direct buckets of ~256 records on average (8 to 12 bits)
    const double est = std::max(1.0, hp_estimate(g, p));
    int db = 8;
    while (db < DX_MAXBITS && est / (double)(1u << db) > g->dx_target) ++db;
    if (g->dx_bits) db = std::min(g->dx_bits, DX_MAXBITS);
    f.dbits = std::min(db, std::max(1, f.wbits + ubits));
    f.dshift = std::max(0, f.wbits + ubits - f.dbits);
  }
  // fixed-capacity buckets: ~CAP/4 records per bucket on average (skew headroom),
  // CAP = 1024 or 2048, at most DX_MAXB buckets
  f.fused = false;
  f.ord11 = false;
  f.caplog = 10;
  if (f.direct && g->fuse_runs) {
    const double est = std::max(1.0, hp_estimate(g, p));
    for (int cl = 10; cl <= 11 && !f.fused; ++cl) {
      int db = 8;
      while (db < DX_MAXBITS && est / (double)(1u << db) > (double)(1u << cl) / 4) ++db;
      if (g->dx_bits) db = std::min(g->dx_bits, DX_MAXBITS);
      db = std::min(db, std::max(1, f.wbits + ubits));
      if (g->dx_bits || est / (double)(1u << db) <= (double)(1u << cl) / 4) {
        const uint64_t slots = (uint64_t)1 << (db + cl);  // candidate slots: one CAP range per bucket
        TRY(wsget(ws, B_SP_BKT, slots * EXB_SUB, &f.bkt));   // record slots: EXB_SUB sub-buckets per bucket
        // the candidate columns are indexed by bucket slot
        TRY(wsget(ws, B_SP_CU, std::max(capW, slots), &f.cu));
        TRY(wsget(ws, B_SP_CW, std::max(capW, slots), &f.cw));
        TRY(wsget(ws, B_SP_CS, std::max(capW, slots), &f.cs));
        TRY(wsget(ws, B_SP_OK0, std::max(capW, slots), &f.ok0));
        TRY(wsget(ws, B_SP_OV0, std::max(capW, slots), &f.ov0));
        TRY(wsget(ws, B_SP_SEGCNT, std::max<uint64_t>((capW + RU_SEG - 1) / RU_SEG + 1, DX_MAXB), &f.segcnt));
        f.fused = true;
        f.ord11 = g->ord11;
        f.caplog = cl;
        f.dbits = db;
        f.dshift = std::max(0, f.wbits + ubits - db);
      }
    }
  }
  // The count metrics do not depend on the order of a run's wedges, so their
  // survivors can come from the degree-class index in any order; Adamic-Adar and
  // Resource-Allocation sum in ascending v and keep the ordered survivor scan.
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  f.dindex = g->use_dindex && !custom && p.H >= 1 && p.H <= DCAP && g->vbydeg;
  f.nv = f.dindex ? g->dstart[p.H + 1] : 0;
  f.survivors = f.dindex ? g->vbydeg : f.surv;
  if (f.dindex && g->use_rindex && (ua > 0 || ub < S)) {  // a shard: its own, smaller index
    nlp_status s = ensure_range_index(g, ua, ub, p.H);
    if (s != NLP_OK) return s;
    f.nv = g->rx_dstart[p.H + 1];
    f.survivors = g->rx_vbydeg;
  }
  const uint64_t tS = (S + SV_TILE - 1) / SV_TILE, tE = (S + NT - 1) / NT;
  const uint64_t tR = std::max<uint64_t>((capW + RN_TILE - 1) / RN_TILE, DX_MAXB);  // also k_sp_grouprun's buckets
  const uint64_t tO = (capW + OS2_TILE - 1) / OS2_TILE;
  f.ostride = tO * RS_BINS;
  {  // counted passes when the candidates may fit CP_MAXT tiles, unless a similar call overflowed.  The
     // estimate is 0.5 sum deg^2 over the survivors scaled by the range's share of the sources: it
     // overstates the candidates (w > u, exclusion, duplicates) and, for the wedge-balanced ranges of
     // a sharded job, can be off by the range's weight -- so try up to 4x the capacity; an overflow
     // (F_CPASS) costs one redo and is remembered
    const double est = hp_estimate(g, p), cap = (double)CP_MAXT * OS2_TILE;
    f.counted = f.fused && !f.ord11 && g->counted && (g->counted_force || est < 4.0 * cap) &&
                !(g->cp_off_w > 0 && est > 0.5 * g->cp_off_w);
    // small calls: one launch ranks every candidate (k_sp_order_rank) when the estimate -- at least
    // the wedges w > u, so at least the candidates -- fits it, unless a similar call did not (F_SMALL)
    f.small = f.fused && !f.ord11 && g->small_order && !g->counted_force &&
              (g->small_force || est <= (double)SO_MAX) && !(g->small_off_w > 0 && est > 0.5 * g->small_off_w);
    if (f.small) f.counted = false;
  }
  f.ostride11 = tO * 2048;
  f.d_tick = SP_DESC;
  f.d_bcur = f.d_tick + SP_NTICK / 2;
  f.d_ts = f.d_bcur + DX_MAXB * EXB_SUB / 2;
  f.d_wsum = f.d_ts + TS_WORDS;
  f.d_surv = f.d_wsum + WSUM_COPIES;
  f.d_exp = f.d_surv + tS + 1;
  f.d_run = f.d_exp + tE + 1;
  f.d_rec = f.d_run + tR + 1;
  f.d_ord = f.d_rec + ((uint64_t)f.passes * f.ostride + 1) / 2;
  f.d_cm = f.d_ord + (std::max(4 * f.ostride, 3 * f.ostride11) + 1) / 2;
  f.arena_words = f.d_cm + 4 * (uint64_t)CP_MAXT * RS_BINS / 2;
  TRY(wsget(ws, B_SP_ARENA, f.arena_words, &f.arena));
  f.zero = ArenaZero{{0, 0, 0}, {f.arena_words, 0, 0}};
  // without the degree-class index k_sp_survivors runs: its look-back
  // descriptors [d_surv, d_exp) are reset with the counters (an earlier call
  // with another survivor set, or a new arena, leaves them dirty)
  const uint64_t zend = f.dindex ? f.d_surv : f.d_exp;
  if (f.fused) f.zero = ArenaZero{{0, SP_HORD, 0}, {SP_HREC, zend, 0}};
  // counted passes: no score-digit histogram copies to reset (the tickets: the survivor scan's)
  if (f.counted) f.zero = ArenaZero{{0, SP_DESC, 0}, {SP_HREC, zend, 0}};
  return NLP_OK;
}

// The stage timed as the dominant kernel by default: the scoring kernel.
int sp_hot_default(const SpBufs& f) {
  const int s_runs = 4 + (f.msd ? f.msd_passes : f.passes) + (f.split ? 1 : 0);
  return f.fused ? s_runs - 1 : s_runs;
}

// Algorithmic bytes of one launch of sort-path stage `s`,
// from the call's own counters (host copy of the arena counters).
uint64_t sp_stage_bytes(const nlp_graph* g, const SpBufs& f, int s, const uint64_t* h, uint32_t H) {
  const uint64_t S = g->span, V = h[C_NV], W = h[C_W], C = h[C_C];
  if (s == 1) return 4 * S + 4 * V;             // deg read, survivor ids written
  if (s == 2 && f.fused && f.dindex && g->sv_pack) {
    // k_sp_exbucket over the degree-class index: survivor id + packed row (and
    // in-row when asymmetric) per survivor, the survivors' lists (P_H =
    // sum of d n_d over 1 <= d <= H; in-lists counted alike), 8-byte records
    uint64_t P = 0;
    for (uint64_t d = 1; d <= H && d < g->deg_hist.size(); ++d) P += d * g->deg_hist[d];
    const uint64_t asym = g->sv_pack_in ? 1 : 0;
    return (12 + 8 * asym) * V + 4 * (1 + asym) * P + 8 * W;
  }
  if (s == 2) return 4 * V + 4 * V + 16 * V + 8 * V + 4 * W + 12 * W;  // ids, deg, toff pair, off, keys, records
  const int P = f.msd ? f.msd_passes : f.passes;
  if (s >= 4 && s < 4 + P) return 24 * W;  // records in + out
  if (f.fused && s == 4 + P) return 8 * W + 4 * ((uint64_t)1 << f.dbits) + 20 * C;  // grouprun: counts + keys in,
                                                                                    // candidates out (u, w, score, key, slot)
  if (f.split && s == 4 + P) return 8 * W + 8 * W + 4 * W;  // bucket sort: keys in, sorted keys + run lengths out
  if (f.split && s == 5 + P) return 8 * W + 4 * W + 20 * C;  // runs: sorted keys, run lengths, candidates
  if (s == 4 + P) return f.msd ? 8 * W + 20 * C : 12 * W + 4 * W + 20 * C;  // records (+stash), candidates
  return 0;
}

// The sort path as an ordered list of stages; seg < 0 launches all stages and
// records the events, seg = 0..3 launches one capture segment:
// [0, hot) | hot | (hot, runs] | (runs, end].
nlp_status launch_sp(nlp_graph* g, const Params& p, const SpBufs& f, EdgeOut* out, hipStream_t st, int seg) {
  const uint64_t S = g->span;
  const uint64_t ua = std::min(p.ua, S), ub = std::min(p.ub, S);
  const uint64_t capW = g->capW;
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  const GraphView gv = view_of(g, p.metric, p.maxf2);
  uint64_t* ctr = f.arena;
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  uint32_t* hrec = (uint32_t*)(f.arena + SP_HREC);
  uint32_t* hord = (uint32_t*)(f.arena + SP_HORD);
  uint32_t* drec = (uint32_t*)(f.arena + f.d_rec);
  uint32_t* dord = (uint32_t*)(f.arena + f.d_ord);
  uint32_t* cmat = (uint32_t*)(f.arena + f.d_cm);  // counted passes: matrix j at cmat + j CP_M
  constexpr uint64_t CP_M = (uint64_t)CP_MAXT * RS_BINS;
  // bucket groups of the counted pass 0 over the buckets that can hold keys
  // (the top bucket bits cover 2^ubits sources, the range only ub - ua of them)
  const uint64_t nb_used = std::min<uint64_t>(
      (uint64_t)1 << f.dbits, (((ub - ua - 1) << f.wbits | ((1ull << f.wbits) - 1)) >> f.dshift) + 1);
  const uint32_t cp_g = (uint32_t)((nb_used + CP_MAXT - 1) / CP_MAXT);        // buckets per group (<= CP_MAXG)
  const uint32_t cp_groups = (uint32_t)((nb_used + cp_g - 1) / cp_g);
  uint32_t* tick = (uint32_t*)(f.arena + f.d_tick);
  uint64_t* ts = f.arena + f.d_ts;
  const int P = f.msd ? f.msd_passes : f.passes;
  const int s_runs = 4 + P + (f.split ? 1 : 0), n_st = s_runs + 7;
  // after the record passes the records sit in buffer 1 for an odd count, 0 for even
  uint64_t* rk_m = (P & 1) ? f.rk1 : f.rk0;
  uint32_t* rv_m = (P & 1) ? f.rv1 : f.rv0;
  uint32_t* rv_free = (P & 1) ? f.rv0 : f.rv1;
  const int hot = g->hot_stage < 0 ? sp_hot_default(f) : std::min(std::max(g->hot_stage, 1), n_st - 1);
  auto grid = [](uint64_t tiles, unsigned occ) {
    return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(tiles, occ)));
  };
  const uint64_t tO = (capW + OS2_TILE - 1) / OS2_TILE;
  // sorted records / candidate order end up in buffer 0 after an even number of passes
  uint64_t* rks = (P & 1) ? f.rk1 : f.rk0;
  uint32_t* rvs = (P & 1) ? f.rv1 : f.rv0;
  auto stage = [&](int s) -> nlp_status {
    if (s == 0) {
      CtrInit ci;
      for (int i = 0; i < NCTR; ++i) ci.v[i] = 0;
      ci.v[C_NV] = f.nv;
      const uint64_t zw = (f.zero.hi[0] - f.zero.lo[0]) + (f.zero.hi[1] - f.zero.lo[1]) + (f.zero.hi[2] - f.zero.lo[2]);
      hipLaunchKernelGGL(k_sp_arena_init, dim3((unsigned)std::min<uint64_t>(1024, (zw + NT - 1) / NT)), dim3(NT), 0, st,
                         f.arena, f.zero, ci);
    } else if (s == 1) {
      if (f.dindex) return NLP_OK;
      hipLaunchKernelGGL(k_sp_survivors, grid((S + SV_TILE - 1) / SV_TILE, g->occ_surv), dim3(NT), 0, st,
                         (const uint32_t*)g->deg, S, p.H, f.surv, f.arena + f.d_surv, tick + TK_SURV, ctr,
                         hot == 1 ? g->d_stamp : nullptr, ts);
    } else if (s == 2) {
      // survivors: known exactly with the degree-class index, else at most S
      const uint64_t nsv = f.dindex ? f.nv : S;
      if (f.fused) {
        const int spt = g->exb_spt;
#define NLP_EXBUCKET(SPT)                                                                                        \
  hipLaunchKernelGGL(k_sp_exbucket<SPT>, dim3((unsigned)std::max<uint64_t>(1, (nsv + NT * SPT - 1) / (NT * SPT))),  \
                     dim3(NT), 0, st, gv, ua, ub, f.wbits, f.survivors, f.dshift, f.dbits, f.caplog, f.bkt,     \
                     (uint32_t*)(f.arena + f.d_bcur), ctr, f.arena + f.d_wsum, ts,                             \
                     (const uint64_t*)(f.survivors == g->vbydeg ? g->sv_pack : nullptr),                         \
                     hot == s ? g->d_stamp : nullptr,                                                           \
                     (const uint64_t*)(f.survivors == g->vbydeg ? g->sv_pack_in : nullptr))
        if (spt >= 4) NLP_EXBUCKET(4);
        else if (spt == 2) NLP_EXBUCKET(2);
        else NLP_EXBUCKET(1);
#undef NLP_EXBUCKET
        TRY(hipGetLastError());
        return NLP_OK;
      }
      if (f.direct) {
        hipLaunchKernelGGL(k_sp_excount, dim3((unsigned)std::max<uint64_t>(1, (nsv + NT - 1) / NT)), dim3(NT), 0, st,
                           gv, ua, ub, f.wbits, f.survivors, ctr, f.dshift, f.dbits, hrec, f.arena + f.d_wsum, ts);
        TRY(hipGetLastError());
        return NLP_OK;
      }
      const int xi = g->ex_ipt;
      const dim3 gx = grid((nsv + (uint64_t)NT * xi - 1) / ((uint64_t)NT * xi), g->occ_exp);
#define NLP_EXPAND(IPT)                                                                                          \
  do {                                                                                                           \
    if (f.msd) /* the MSD digit histogram is fused into the expansion */                                         \
      hipLaunchKernelGGL((k_sp_expand<true, IPT>), gx, dim3(NT), 0, st, gv, ua, ub, f.wbits, f.survivors, capW,  \
                         f.rk0, f.rv0, f.arena + f.d_exp, tick + TK_EXP, ctr, f.msd_shift, hrec, P, ts);         \
    else                                                                                                         \
      hipLaunchKernelGGL((k_sp_expand<false, IPT>), gx, dim3(NT), 0, st, gv, ua, ub, f.wbits, f.survivors, capW, \
                         f.rk0, f.rv0, f.arena + f.d_exp, tick + TK_EXP, ctr, 0, (uint32_t*)nullptr, 1, ts);     \
  } while (0)
      if (xi == 4) NLP_EXPAND(4);
      else if (xi == 2) NLP_EXPAND(2);
      else NLP_EXPAND(1);
#undef NLP_EXPAND
    } else if (s == 3) {
      if (f.fused) return NLP_OK;  // k_sp_exbucket placed the records
      if (f.direct) {  // records straight into their MSD buckets (the buffers the bucket sort reads)
        const uint64_t nsv = f.dindex ? f.nv : S;
        hipLaunchKernelGGL(k_sp_exemit, dim3((unsigned)std::max<uint64_t>(1, (nsv + NT - 1) / NT)), dim3(NT), 0, st,
                           gv, ua, ub, f.wbits, f.survivors, capW, rk_m, rv_m, ctr, f.dshift, f.dbits,
                           (const uint32_t*)hrec, (uint32_t*)(f.arena + f.d_bcur),
                           (const uint64_t*)(f.arena + f.d_wsum));
        TRY(hipGetLastError());
        return NLP_OK;
      }
      if (f.msd) return NLP_OK;
      hipLaunchKernelGGL(k_sp_hist<uint64_t>, dim3(128), dim3(NT), 0, st, (const uint64_t*)f.rk0,
                         (const uint64_t*)&ctr[C_W], capW, f.msd ? f.msd_shift : 0, P, hrec, &ctr[C_WSORT],
                         &ctr[C_FLAGS]);
    } else if (s < 4 + P) {
      if (f.direct) return NLP_OK;  // the records are already in their buckets
      const int ps = s - 4;
      const bool odd = ps & 1;
      hipLaunchKernelGGL((k_sp_pass<uint64_t, OS2_IPT>), grid(tO, g->occ_p64), dim3(OS_NT), 0, st,
                         (const uint64_t*)(odd ? f.rk1 : f.rk0), (const uint32_t*)(odd ? f.rv1 : f.rv0),
                         odd ? f.rk0 : f.rk1, odd ? f.rv0 : f.rv1, (const uint64_t*)&ctr[C_WSORT],
                         f.msd ? f.msd_shift + 8 * ps : 8 * ps,
                         (const uint32_t*)(hrec + ps * RS_BINS), drec + (uint64_t)ps * f.ostride, tick + TK_REC + ps,
                         err, hot == s ? g->d_stamp : nullptr, GatherOut{}, (uint32_t*)nullptr);
    } else if (f.split && s == s_runs - 1 && P == 1 && g->group_sort != 1 && !f.direct) {
      // one MSD pass: one workgroup per top-digit bucket, the bucket bounds from its histogram
      if (custom)
        hipLaunchKernelGGL((k_sp_bucket<true, true>), dim3(RS_BINS), dim3(BK_NT), 0, st, gv, p.metric, p.min_score, ua,
                           f.wbits, (const uint64_t*)rk_m, (const uint32_t*)rv_m, (const uint32_t*)hrec, f.cu, f.cw,
                           f.cs, f.ok0, f.ov0, f.arena + f.d_run, ctr, f.msd_shift, p.max_edges, hord,
                           hot == s ? g->d_stamp : nullptr, rk_m, rv_free, (uint32_t*)f.stash);
      else
        hipLaunchKernelGGL((k_sp_bucket<false, true>), dim3(RS_BINS), dim3(BK_NT), 0, st, gv, p.metric, p.min_score,
                           ua, f.wbits, (const uint64_t*)rk_m, (const uint32_t*)rv_m, (const uint32_t*)hrec, f.cu,
                           f.cw, f.cs, f.ok0, f.ov0, f.arena + f.d_run, ctr, f.msd_shift, p.max_edges, hord,
                           hot == s ? g->d_stamp : nullptr, rk_m, rv_free, (uint32_t*)nullptr);
    } else if (f.split && s == s_runs - 1) {
      const dim3 gr((unsigned)std::max<uint64_t>(1, (capW + GR_T - 1) / GR_T));
      if (f.fused) {
        const uint32_t nb = 1u << f.dbits;
#define NLP_GROUPRUN3(CL, DB, NTH)                                                                               \
  hipLaunchKernelGGL((k_sp_grouprun<CL, DB, NTH>), dim3(nb), dim3(NTH), 0, st, gv, p.metric, p.min_score, ua,      \
                     f.wbits,                                                                                    \
                     (const uint64_t*)f.bkt, (const uint32_t*)(f.arena + f.d_bcur), f.cu, f.cw, f.cs, f.ok0,    \
                     f.ov0, f.segcnt, ctr, f.counted ? cmat : hord, (const uint64_t*)(f.arena + f.d_wsum),    \
                     hot == s ? g->d_stamp : nullptr, ts, f.counted ? cp_g : 0u)
#define NLP_GROUPRUN(CL, DB)                \
  do {                                      \
    if (g->gr_nt == 512)                    \
      NLP_GROUPRUN3(CL, DB, 512);           \
    else                                    \
      NLP_GROUPRUN3(CL, DB, GR_NT);         \
  } while (0)
        if (f.caplog == 11 && f.ord11) NLP_GROUPRUN(11, 11);
        else if (f.caplog == 11) NLP_GROUPRUN(11, 8);
        else if (f.ord11) NLP_GROUPRUN(10, 11);
        else NLP_GROUPRUN(10, 8);
#undef NLP_GROUPRUN
#undef NLP_GROUPRUN3
      }
      else if (custom)
        hipLaunchKernelGGL(k_sp_group<true>, gr, dim3(BK_NT), 0, st, (const uint64_t*)rk_m, (const uint32_t*)rv_m,
                           f.msd_shift, rk_m, rv_free, (uint32_t*)f.stash, ctr, hot == s ? g->d_stamp : nullptr);
      else  // after direct emission the fine buckets are the dbits-bit buckets
        hipLaunchKernelGGL(k_sp_group<false>, gr, dim3(BK_NT), 0, st, (const uint64_t*)rk_m, (const uint32_t*)rv_m,
                           f.direct ? f.dshift : f.msd_shift, rk_m, rv_free, (uint32_t*)nullptr, ctr,
                           hot == s ? g->d_stamp : nullptr);
    } else if (f.split && s == s_runs) {
      if (f.fused) return NLP_OK;  // scored by k_sp_grouprun
      // one workgroup per RU_TILE records, no hand-off (gapped output)
      const dim3 gr((unsigned)std::max<uint64_t>(1, (capW + RU_TILE - 1) / RU_TILE));
      if (custom)
        hipLaunchKernelGGL(k_sp_runs<true>, gr, dim3(NT), 0, st, gv, p.metric, p.min_score, ua, f.wbits,
                           (const uint64_t*)rk_m, (const uint32_t*)rv_free, (const uint32_t*)f.stash, f.cu, f.cw,
                           f.cs, f.ok0, f.ov0, f.segcnt, ctr, hord, hot == s ? g->d_stamp : nullptr, ts);
      else
        hipLaunchKernelGGL(k_sp_runs<false>, gr, dim3(NT), 0, st, gv, p.metric, p.min_score, ua, f.wbits,
                           (const uint64_t*)rk_m, (const uint32_t*)rv_free, (const uint32_t*)nullptr, f.cu, f.cw,
                           f.cs, f.ok0, f.ov0, f.segcnt, ctr, hord, hot == s ? g->d_stamp : nullptr, ts);
    } else if (s == s_runs && f.msd) {
      if (custom)
        hipLaunchKernelGGL(k_sp_bucket<true>, dim3(RS_BINS), dim3(BK_NT), 0, st, gv, p.metric, p.min_score, ua,
                           f.wbits, (const uint64_t*)f.rk1, (const uint32_t*)f.rv1, (const uint32_t*)hrec, f.cu,
                           f.cw, f.cs, f.ok0, f.ov0, f.arena + f.d_run, ctr, f.msd_shift, p.max_edges, hord,
                           hot == s ? g->d_stamp : nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                           (uint32_t*)nullptr, tick + TK_BUCKET);
      else
        hipLaunchKernelGGL(k_sp_bucket<false>, dim3(RS_BINS), dim3(BK_NT), 0, st, gv, p.metric, p.min_score, ua,
                           f.wbits, (const uint64_t*)f.rk1, (const uint32_t*)f.rv1, (const uint32_t*)hrec, f.cu,
                           f.cw, f.cs, f.ok0, f.ov0, f.arena + f.d_run, ctr, f.msd_shift, p.max_edges, hord,
                           hot == s ? g->d_stamp : nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                           (uint32_t*)nullptr, tick + TK_BUCKET);
    } else if (s == s_runs) {
      const dim3 gr = grid((capW + RN_TILE - 1) / RN_TILE, g->occ_run);
      if (custom) {
        F_Runs<true> fr{gv, p.metric, p.min_score, ua, f.wbits, rks, rvs, f.stash, f.cu, f.cw, f.cs, f.ok0, f.ov0,
                        &ctr[C_NAN]};
        hipLaunchKernelGGL((k_sp_scan<F_Runs<true>, RN_IPT>), gr, dim3(NT), 0, st, fr, (const uint64_t*)&ctr[C_WSORT],
                           f.arena + f.d_run, tick + TK_RUNS, err, &ctr[C_C]);
      } else {
        F_Runs<false> fr{gv, p.metric, p.min_score, ua, f.wbits, rks, rvs, f.stash, f.cu, f.cw, f.cs, f.ok0, f.ov0,
                         &ctr[C_NAN]};
        hipLaunchKernelGGL((k_sp_scan<F_Runs<false>, RN_IPT>), gr, dim3(NT), 0, st, fr,
                           (const uint64_t*)&ctr[C_WSORT], f.arena + f.d_run, tick + TK_RUNS, err, &ctr[C_C]);
      }
    } else if (s == s_runs + 1) {
      if (f.msd) return NLP_OK;  // fused into k_sp_bucket
      hipLaunchKernelGGL(k_sp_hist<uint32_t>, dim3(128), dim3(NT), 0, st, (const uint32_t*)f.ok0,
                         (const uint64_t*)&ctr[C_C], capW, 0, 4, hord, (uint64_t*)nullptr, (uint64_t*)nullptr);
    } else if (s < s_runs + 6) {
      const int ps = s - (s_runs + 2);
      const bool odd = ps & 1;
      if (f.small) {  // all four passes and the output in one launch (rank by counting)
        if (ps != 0) return NLP_OK;
        hipLaunchKernelGGL(k_sp_order_rank, dim3(SR_GRID), dim3(OS_NT), 0, st, (const uint32_t*)f.ok0,
                           (const uint32_t*)f.cu, (const uint32_t*)f.cw, (const float*)f.cs, (const uint32_t*)f.segcnt,
                           (uint32_t)nb_used, f.caplog,
                           GatherOut{nullptr, nullptr, nullptr, p.max_edges, out, ctr, g->host_ctr_dev, ts, g->d_sticky},
                           ts + TS_HOT_OUT, hot == s ? g->d_stamp : nullptr);
      } else if (f.counted && ps == 0) {  // dense tiles of k_sp_grouprun's candidates (it counted digit 0 per bucket group)
        hipLaunchKernelGGL(k_sp_cpass0, dim3(CP_MAXT), dim3(OS_NT), 0, st, (const uint32_t*)f.ok0,
                           (const uint32_t*)f.cu, (const uint32_t*)f.cw, (const float*)f.cs, (const uint32_t*)f.segcnt,
                           (uint32_t)nb_used, cp_g, cp_groups, f.caplog, (const uint32_t*)cmat, cmat + CP_M, f.ok1,
                           (uint64_t*)f.rk0, f.ov1, ctr, ts + TS_HOT_OUT, hot == s ? g->d_stamp : nullptr);
      } else if (f.counted) {  // pass ps from matrix ps; cleans matrix ps - 1
        const uint32_t* m_in = cmat + (uint64_t)ps * CP_M;
        uint32_t* const m_old = cmat + (uint64_t)(ps - 1) * CP_M;
        const uint32_t rows_old = ps == 1 ? cp_groups : 0u;  // matrix 0 has a row per bucket group
        const uint32_t words_old = ps == 1 ? RS_BINS : RS_BINS / 2;  // u32 counts; matrices 1-3 u16 pairs
        // matrix 3 (read by every tile of the last pass, so not cleaned there) is zeroed by pass 1
        uint32_t* const m_last = ps == 1 ? cmat + 3 * CP_M : nullptr;
        // payload ping-pong: A = (ok1, rk0, ov1) after passes 0 and 2, B = (ok0, rk1, ov0) after pass 1
        const uint32_t* kA = f.ok1; const uint64_t* uwA = (const uint64_t*)f.rk0; const uint32_t* sA = f.ov1;
        if (ps == 1)
          hipLaunchKernelGGL(k_sp_cpass<true>, dim3(CP_MAXT), dim3(OS_NT), 0, st, kA, uwA, sA, f.ok0,
                             (uint64_t*)f.rk1, f.ov0, (const uint64_t*)&ctr[C_C], 8, m_in, cmat + 2 * CP_M, m_old,
                             rows_old, words_old, hot == s ? g->d_stamp : nullptr, GatherOut{}, m_last);
        else if (ps == 2)
          hipLaunchKernelGGL(k_sp_cpass<true>, dim3(CP_MAXT), dim3(OS_NT), 0, st, (const uint32_t*)f.ok0,
                             (const uint64_t*)f.rk1, (const uint32_t*)f.ov0, f.ok1, (uint64_t*)f.rk0, f.ov1,
                             (const uint64_t*)&ctr[C_C], 16, m_in, cmat + 3 * CP_M, m_old, rows_old, words_old,
                             hot == s ? g->d_stamp : nullptr, GatherOut{});
        else  // the last pass writes the caller's edges and publishes the counters
          hipLaunchKernelGGL((k_sp_cpass<false, true>), dim3(CP_MAXT), dim3(OS_NT), 0, st, kA, uwA, sA,
                             (uint32_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr, (const uint64_t*)&ctr[C_C], 24,
                             m_in, (uint32_t*)nullptr, m_old, rows_old, words_old, hot == s ? g->d_stamp : nullptr,
                             GatherOut{nullptr, nullptr, nullptr, p.max_edges, out, ctr, g->host_ctr_dev, ts, g->d_sticky});
      } else if (f.fused && !f.ord11 && ps == 0)  // k_sp_grouprun's per-bucket candidates (it counted digit 0); this pass counts 1-3
        hipLaunchKernelGGL((k_sp_pass<uint32_t, OS2_IPT, false, true, GAP_BUCKETS>), grid(tO, g->occ_p32),
                           dim3(OS_NT), 0, st, (const uint32_t*)f.ok0, (const uint32_t*)f.ov0, f.ok1, f.ov1,
                           (const uint64_t*)&ctr[C_C], 0, (const uint32_t*)hord, dord, tick + TK_ORD, err,
                           hot == s ? g->d_stamp : nullptr, GatherOut{}, hord + RS_BINS, (const uint32_t*)f.segcnt,
                           &ctr[C_C], (const uint64_t*)nullptr, 1u << f.dbits, f.caplog, ts + TS_HOT_OUT);
      else if (f.fused && ps == 0)  // the same with 11-bit digits; this pass counts digits 1-2
        hipLaunchKernelGGL((k_sp_pass<uint32_t, OS2_IPT, false, true, GAP_BUCKETS, 11>), grid(tO, g->occ_p11),
                           dim3(OS_NT), 0, st, (const uint32_t*)f.ok0, (const uint32_t*)f.ov0, f.ok1, f.ov1,
                           (const uint64_t*)&ctr[C_C], 0, (const uint32_t*)hord, dord, tick + TK_ORD, err,
                           hot == s ? g->d_stamp : nullptr, GatherOut{}, hord + 2048, (const uint32_t*)f.segcnt,
                           &ctr[C_C], (const uint64_t*)nullptr, 1u << f.dbits, f.caplog, ts + TS_HOT_OUT);
      else if (f.fused && f.ord11 && ps < 3)  // 11-bit digits 1 and 2 (bits 11-21, 22-31)
        hipLaunchKernelGGL((k_sp_pass<uint32_t, OS2_IPT, false, false, GAP_NONE, 11>), grid(tO, g->occ_p11),
                           dim3(OS_NT), 0, st, (const uint32_t*)(ps == 1 ? f.ok1 : f.ok0),
                           (const uint32_t*)(ps == 1 ? f.ov1 : f.ov0), ps == 1 ? f.ok0 : f.ok1,
                           ps == 1 ? f.ov0 : f.ov1, (const uint64_t*)&ctr[C_C], 11 * ps,
                           (const uint32_t*)(hord + 2048 * ps), dord + (uint64_t)ps * f.ostride11, tick + TK_ORD + ps,
                           err, hot == s ? g->d_stamp : nullptr, GatherOut{}, (uint32_t*)nullptr,
                           (const uint32_t*)nullptr, (uint64_t*)nullptr, (const uint64_t*)nullptr, 0u, 0,
                           (uint64_t*)nullptr, dord + (uint64_t)(ps - 1) * f.ostride11);
      else if (f.fused && f.ord11)
        return NLP_OK;  // three 11-bit passes
      else if (f.split && ps == 0)  // k_sp_runs' gapped candidates (and digit 0); this pass counts digits 1-3
        hipLaunchKernelGGL((k_sp_pass<uint32_t, OS2_IPT, false, true, GAP_SEGMENTS>), grid(tO, g->occ_p32), dim3(OS_NT), 0, st,
                           (const uint32_t*)f.ok0, (const uint32_t*)f.ov0, f.ok1, f.ov1,
                           (const uint64_t*)&ctr[C_WSORT], 0, (const uint32_t*)hord, dord, tick + TK_ORD, err,
                           hot == s ? g->d_stamp : nullptr, GatherOut{}, hord + RS_BINS, (const uint32_t*)f.segcnt,
                           &ctr[C_C], (const uint64_t*)&ctr[C_FLAGS], 0u, 0, ts + TS_HOT_OUT);
      else if (f.msd && ps == 0)  // k_sp_bucket counted digit 0; this pass counts digits 1-3
        hipLaunchKernelGGL((k_sp_pass<uint32_t, OS2_IPT, false, true>), grid(tO, g->occ_p32), dim3(OS_NT), 0, st,
                           (const uint32_t*)f.ok0, (const uint32_t*)f.ov0, f.ok1, f.ov1, (const uint64_t*)&ctr[C_C],
                           0, (const uint32_t*)hord, dord, tick + TK_ORD, err, (uint64_t*)nullptr, GatherOut{},
                           hord + RS_BINS);
      else if (ps == 3 && g->fuse_gather && !f.fused)  // the last pass writes the caller's edges
        hipLaunchKernelGGL((k_sp_pass<uint32_t, OS2_IPT, true>), grid(tO, g->occ_p32), dim3(OS_NT), 0, st,
                           (const uint32_t*)f.ok1, (const uint32_t*)f.ov1, f.ok0, f.ov0, (const uint64_t*)&ctr[C_C], 24,
                           (const uint32_t*)(hord + 3 * RS_BINS), dord + 3 * f.ostride, tick + TK_ORD + 3, err,
                           (uint64_t*)nullptr,
                           GatherOut{f.cu, f.cw, f.cs, p.max_edges, out, ctr, g->host_ctr_dev, ts, g->d_sticky},
                           (uint32_t*)nullptr);
      else
        hipLaunchKernelGGL((k_sp_pass<uint32_t, OS2_IPT>), grid(tO, g->occ_p32), dim3(OS_NT), 0, st,
                           (const uint32_t*)(odd ? f.ok1 : f.ok0), (const uint32_t*)(odd ? f.ov1 : f.ov0),
                           odd ? f.ok0 : f.ok1, odd ? f.ov0 : f.ov1, (const uint64_t*)&ctr[C_C], 8 * ps,
                           (const uint32_t*)(hord + ps * RS_BINS), dord + (uint64_t)ps * f.ostride, tick + TK_ORD + ps,
                           err, hot == s ? g->d_stamp : nullptr, GatherOut{}, (uint32_t*)nullptr,
                           (const uint32_t*)nullptr, (uint64_t*)nullptr, (const uint64_t*)nullptr, 0u, 0,
                           (uint64_t*)nullptr, f.fused ? dord + (uint64_t)(ps - 1) * f.ostride : (uint32_t*)nullptr);
    } else {
      if ((g->fuse_gather && !f.fused) || f.counted || f.small) return NLP_OK;  // done by the last ordering pass
      const uint64_t m = std::min<uint64_t>(p.max_edges, capW);
      // one workgroup per CU at most: the last one to finish is found with one atomic each
      hipLaunchKernelGGL(k_sp_gather, dim3((unsigned)std::min<uint64_t>(256, std::max<uint64_t>(1, (m + NT - 1) / NT))),
                         dim3(NT), 0, st, (const uint32_t*)(f.ord11 ? f.ov1 : f.ov0), (const uint32_t*)f.cu,
                         (const uint32_t*)f.cw, (const float*)f.cs, p.max_edges, out, ctr, g->host_ctr_dev,
                         (const uint64_t*)ts,
                         f.fused ? (f.ord11 ? dord + 2 * f.ostride11 : dord + 3 * f.ostride) : (uint32_t*)nullptr,
                         f.ord11 ? 2048u : (uint32_t)RS_BINS, g->d_sticky);
    }
    TRY(hipGetLastError());
    return NLP_OK;
  };
  // three segments [0, hot) | hot | (hot, end) with events 0, 3, 4 before them
  // and 2 at the end; with the default hot stage (the scoring kernel) event 4
  // also splits scoring from selection
  const int lo[3] = {0, hot, hot + 1}, hi[3] = {hot, hot + 1, n_st};
  static const int ev_at[3] = {0, 3, 4};
  // seg -1: direct launch with event records (captured segments carry none);
  // seg -2: direct launch without events (stamp-timed, the host polls the stream)
  auto mark = [&](int e) -> hipError_t { return seg == -1 ? hipEventRecord(g->ev[e], st) : hipSuccess; };
  if (seg == -2) seg = -3;  // every segment, no marks
  for (int sg = 0; sg < 3; ++sg) {
    if (seg >= 0 && seg != sg) continue;
    TRY(mark(ev_at[sg]));
    for (int s = lo[sg]; s < hi[sg]; ++s) {
      nlp_status r = stage(s);
      if (r != NLP_OK) return r;
    }
  }
  TRY(mark(2));
  return NLP_OK;
}

// Replay (or capture, then replay) a fast path as hipGraphs.  The pipeline is
// captured as four segments on the graph's own stream and replayed on the
// caller's stream with the timing events recorded between them (events inside
// a graph cannot be timed), so hot_ms stays a live measurement.  *replayed =
// false when graphs are disabled or capture failed (the caller then launches
// directly).  launch(stream, seg) enqueues one segment.
// events recorded before each capture segment (event 2 ends the call)
static const int EV_SEG4[4] = {0, 3, 4, 1};  // bucket grouping: pre | hot | rest of scoring | selection
static const int EV_SEG3[3] = {0, 3, 4};     // sort grouping: pre | hot (scoring) | selection

// copy_src: the device counters the pipeline copies to host_small at its end.
// stamps: the hot kernel times itself (sortpath.hpp ts_enter): no event-record
// nodes between the segments of the single graph, only at its start and end.
template <class L>
nlp_status run_graph(nlp_graph* g, const Params& p, EdgeOut* out, hipStream_t st, int mode, const void* copy_src,
                     bool* replayed, L&& launch, bool stamps = false, bool seq_end = false) {
  *replayed = false;
  if (!g->use_graphs) return NLP_OK;
  const bool single = g->graph_single && mode != 0;  // the bucket grouping is captured in segments
  const uint64_t gen = ws_fingerprint(g->ws);
  nlp_graph::Cached* hit = nullptr;
  for (auto& c : g->graphs)
    if (c.metric == p.metric && c.H == p.H && c.min_score == p.min_score && c.max_edges == p.max_edges &&
        c.ua == p.ua && c.ub == p.ub && c.capW == g->capW && c.gen == gen && c.maxf2 == p.maxf2 && c.mode == mode &&
        c.out == (void*)out)
      hit = &c;
  if (!hit) {
    nlp_graph::Cached c{p.metric, p.H,  p.min_score, p.max_edges, p.ua,  p.ub, g->capW,
                        gen,      p.maxf2, mode,   (void*)out,  {},    false, 0};
    hipStream_t gs = g->stream;
    bool ok = true;
    c.single = false;
    hipGraph_t seg_graph[4] = {};
    const int nseg = mode == 0 ? 4 : 3;
    const int* ev_before = mode == 0 ? EV_SEG4 : EV_SEG3;
    for (int seg = 0; seg < nseg && ok; ++seg) {
      if (hipStreamBeginCapture(gs, hipStreamCaptureModeThreadLocal) != hipSuccess) { ok = false; break; }
      nlp_status s = launch(gs, seg);
      hipError_t e = hipStreamEndCapture(gs, &seg_graph[seg]);
      ok = s == NLP_OK && e == hipSuccess && seg_graph[seg];
      if (!ok && debug_on())
        fprintf(stderr, "nlp: graph capture failed (seg=%d launch=%d end=%s)\n", seg, (int)s, hipGetErrorString(e));
    }
    if (ok && single) {
      // One flat graph: the segments' kernel nodes copied in order with
      // event-record nodes between them, so a call is a single launch and the
      // events still time the hot kernel.  (Child-graph nodes would work too but
      // cost several microseconds per boundary.)  The segments are linear
      // chains of kernel nodes plus the final counter copy, which is re-added.
      hipGraph_t top = nullptr;
      bool ok1 = hipGraphCreate(&top, 0) == hipSuccess;
      hipGraphNode_t prev = nullptr;
      auto link = [&](hipGraphNode_t n) { prev = n; };
      auto chain_ev = [&](int e) {
        hipGraphNode_t n = nullptr;
        ok1 = ok1 && hipGraphAddEventRecordNode(&n, top, prev ? &prev : nullptr, prev ? 1 : 0, g->gev[e]) == hipSuccess;
        link(n);
      };
      bool saw_copy = false;
      auto append = [&](hipGraph_t sg) {
        size_t nr = 0;
        ok1 = ok1 && hipGraphGetRootNodes(sg, nullptr, &nr) == hipSuccess;
        if (!ok1 || nr == 0) return;
        if (nr != 1) { ok1 = false; return; }
        hipGraphNode_t node = nullptr;
        ok1 = hipGraphGetRootNodes(sg, &node, &nr) == hipSuccess;
        while (ok1 && node) {
          hipGraphNodeType ty;
          ok1 = hipGraphNodeGetType(node, &ty) == hipSuccess;
          if (!ok1) break;
          if (ty == hipGraphNodeTypeKernel) {
            hipKernelNodeParams kp;
            hipGraphNode_t n = nullptr;
            ok1 = hipGraphKernelNodeGetParams(node, &kp) == hipSuccess &&
                  hipGraphAddKernelNode(&n, top, prev ? &prev : nullptr, prev ? 1 : 0, &kp) == hipSuccess;
            link(n);
          } else if (ty == hipGraphNodeTypeMemcpy) {
            saw_copy = true;  // the counter copy, re-added at the end
          } else {
            ok1 = false;
            break;
          }
          size_t nd = 0;
          ok1 = ok1 && hipGraphNodeGetDependentNodes(node, nullptr, &nd) == hipSuccess;
          if (!ok1 || nd == 0) break;
          if (nd != 1) { ok1 = false; break; }
          ok1 = hipGraphNodeGetDependentNodes(node, &node, &nd) == hipSuccess;
        }
      };
      for (int seg = 0; seg < nseg && ok1; ++seg) {
        if (!stamps) chain_ev(ev_before[seg]);  // stamps: the kernels time the call themselves
        append(seg_graph[seg]);
      }
      if (ok1 && saw_copy) {
        hipGraphNode_t n = nullptr;
        ok1 = hipGraphAddMemcpyNode1D(&n, top, prev ? &prev : nullptr, prev ? 1 : 0, g->host_small, copy_src,
                                      NCTR * 8, hipMemcpyDeviceToHost) == hipSuccess;
        link(n);
      }
      if (ok1 && !seq_end) {  // seq_end: the host polls the stream instead
        if (stamps && g->end_mode == 1) {
          hipGraphNode_t n = nullptr;
          ok1 = hipGraphAddEventRecordNode(&n, top, prev ? &prev : nullptr, prev ? 1 : 0, g->gev_end) == hipSuccess;
          link(n);
        } else if (!(stamps && g->end_mode == 2)) {
          chain_ev(2);
        }
      }
      if (ok1) ok1 = hipGraphInstantiate(&c.exec[0], top, nullptr, nullptr, 0) == hipSuccess;
      if (ok1) (void)hipGraphUpload(c.exec[0], st);  // stage the executable graph on the device once
      if (top) (void)hipGraphDestroy(top);
      if (ok1) {
        c.single = true;
      } else {
        if (c.exec[0]) (void)hipGraphExecDestroy(c.exec[0]);
        c.exec[0] = nullptr;
        (void)hipGetLastError();
        g->graph_single = false;
        if (debug_on()) fprintf(stderr, "nlp: single-graph composition failed, using segments\n");
      }
    }
    for (int seg = 0; seg < nseg && ok && !c.single; ++seg) {
      hipError_t ei = hipGraphInstantiate(&c.exec[seg], seg_graph[seg], nullptr, nullptr, 0);
      ok = ei == hipSuccess;
    }
    for (auto& x : seg_graph)
      if (x) (void)hipGraphDestroy(x);
    if (!ok) {
      for (auto& x : c.exec)
        if (x) (void)hipGraphExecDestroy(x);
      (void)hipGetLastError();
      g->use_graphs = false;
      return NLP_OK;
    }
    if (g->graphs.size() >= 32) {  // evict the least recently used
      size_t lru = 0;
      for (size_t i = 1; i < g->graphs.size(); ++i)
        if (g->graphs[i].last_use < g->graphs[lru].last_use) lru = i;
      for (auto& x : g->graphs[lru].exec)
        if (x) (void)hipGraphExecDestroy(x);
      g->graphs.erase(g->graphs.begin() + lru);
    }
    g->graphs.push_back(c);
    hit = &g->graphs.back();
  }
  hit->last_use = ++g->use_clock;
  g->last_single = hit->single;
  if (hit->single) {
    TRY(hipGraphLaunch(hit->exec[0], st));
    if (stamps && !seq_end && g->end_mode == 2) TRY(hipEventRecord(g->gev_end, st));
  } else {
    const int nseg = mode == 0 ? 4 : 3;
    const int* ev_before = mode == 0 ? EV_SEG4 : EV_SEG3;
    for (int seg = 0; seg < nseg; ++seg) {
      TRY(hipEventRecord(g->ev[ev_before[seg]], st));
      TRY(hipGraphLaunch(hit->exec[seg], st));
    }
    TRY(hipEventRecord(g->ev[2], st));
  }
  *replayed = true;
  return NLP_OK;
}

// Run the fast path; *handled = false when the caller must use the general
// flow (wedges beyond the budget, or -- bucket grouping -- a bucket beyond the
// LDS cap).
// hprof (build-time): host-side phase times of the fast path, averaged and printed
// every 100 calls (diagnostics of the per-call overhead outside the kernels).
struct HostProf {
  double prep = 0, launch = 0, wait = 0, post = 0;
  int n = 0;
};
inline double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void async_key_of(const Params& p, uint64_t (&k)[6]) {
  uint32_t ms;
  memcpy(&ms, &p.min_score, 4);
  k[0] = (uint64_t)(uint32_t)p.metric | (uint64_t)p.H << 32;
  k[1] = (uint64_t)p.maxf2 | (uint64_t)ms << 32;
  k[2] = p.max_edges;
  k[3] = p.ua;
  k[4] = p.ub;
  k[5] = 0;
}

// Timing of a stamp-timed single-graph call from its published stamps (10 ns
// ticks): first kernel entry, hot kernel entry and end, the end of the call.
void stamp_times(const uint64_t* h, float* score, float* select, float* hot) {
  const uint64_t* ts = h + NCTR;
  const float tot = ts[TS_END] > ~ts[TS_FIRST] ? (float)((ts[TS_END] - ~ts[TS_FIRST]) * 1e-5) : 0.0f;
  *hot = ts[TS_HOT_OUT] > ~ts[TS_HOT_IN] ? (float)((ts[TS_HOT_OUT] - ~ts[TS_HOT_IN]) * 1e-5) : 0.0f;
  float a = ts[TS_HOT_OUT] > ~ts[TS_FIRST] ? (float)((ts[TS_HOT_OUT] - ~ts[TS_FIRST]) * 1e-5) : 0.0f;
  a = std::min(a, tot);
  *score = a;
  *select = tot - a;
}

// async: enqueue only (nlp_predict_device_async) -- the caller checked that the
// same call last ran synchronously on its first attempt as a replayed graph;
// the call's flags reach g->d_sticky, its counters and stamps host_ctr.
nlp_status predict_fast(nlp_graph* g, const Params& p, EdgeOut* d_out, uint64_t* out_count, nlp_timing* t,
                        hipStream_t st, EdgeOut** result, bool* handled, bool async = false) {
  constexpr bool hprof = false;  // host-side phase times of the fast path (a build-time diagnostic)
  static HostProf hp;
  double t0 = hprof ? now_us() : 0, t1 = 0, t2 = 0, t3 = 0;
  *handled = false;
  const bool sorted = g->sort_grouping;
  bool msd = !g->sort_lsd;  // sort grouping: MSD bucket kernel first, full LSD sort when a bucket is too big
  // MSD passes: fine buckets of about a thousand records on average, from the
  // wedge count of the previous call (one more pass, then the full LSD sort,
  // when a fine bucket is still above the LDS capacity)
  int msd_passes = g->last_wedges > (256u << 10) ? 2 : 1;
  // start from the grouping that succeeded last time for a similar wedge count
  // (each failed attempt costs a full pipeline run)
  const double est_w = hp_estimate(g, p);
  if (msd && g->last_ok_w > 0 && est_w < 2.0 * (double)g->last_ok_w && est_w > 0.5 * (double)g->last_ok_w) {
    msd = g->last_ok_msd;
    msd_passes = g->last_ok_passes;
  }
  if (g->msd_force) {
    msd = true;
    msd_passes = g->msd_force;
  }
  // size the record buffers from the wedge estimate up front (an overflow costs a rerun)
  if (sorted) {
    const double est = est_w;
    if (est * 1.1 > (double)g->capW && est * 1.1 < (double)SP_MAX_N) g->capW = (uint64_t)(est * 1.1) + 1024;
  }
  for (int attempt = 0; attempt < 4; ++attempt) {
    if (sorted && g->capW > SP_MAX_N) return NLP_OK;
    EdgeOut* out = d_out;
    if (!out) TRY(wsget(g->ws, B_EDGES, std::max<uint64_t>(std::min(p.max_edges, g->capW), 1), &out));
    FastBufs f;
    SpBufs sp;
    nlp_status s = sorted ? prepare_sp(g, p, sp, msd, msd_passes) : prepare_fast(g, p, f, st);
    if (s != NLP_OK) return s;
    // the fused path leaves its ordering descriptors zero; after any other call
    // (or a new arena) they are zeroed here, outside the captured pipeline
    if (sorted && sp.fused && g->ord_clean != sp.arena)
      TRY(hipMemsetAsync(sp.arena + sp.d_ord, 0, (sp.arena_words - sp.d_ord) * sizeof(uint64_t), st));
    g->ord_clean = nullptr;
    bool replayed = false;
    g->last_single = false;
    if (hprof) t1 = now_us();
    const bool stamps = sorted && sp.split && g->hot_stage < 0;
    // Stamp-timed graphs end without an event node and the host polls the
    // stream (an end event instead measured equal).  Equal for one
    // synchronous call; back-to-back calls (nlp_predict_device_async) run
    // 0.117 -> 0.111 ms each on C2, the event node costing GPU time per graph.
    constexpr bool stream_wait = true;
    const bool gseq = stream_wait && sorted;
    // asynchronous stamp-timed calls are launched kernel by kernel (below): the
    // host's ~40 us of launches hide behind the previous call's kernels, and
    // back-to-back graph launches leave ~10 us between graphs on the GPU
    // (C2: 0.101 vs 0.109 ms per call)
    const bool async_direct = stamps && ((async && g->async_direct) || (!async && g->sync_direct));
    if (sorted && async_direct)
      replayed = false;
    else if (sorted)
      s = run_graph(g, p, out, st, (msd ? 1 + sp.msd_passes : 1) + (sp.counted ? 16 : 0) + (sp.small ? 32 : 0), sp.arena, &replayed,
                    [&](hipStream_t gs, int seg) { return launch_sp(g, p, sp, out, gs, seg); }, stamps,
                    stamps && gseq);
    else
      s = run_graph(g, p, out, st, 0, f.arena, &replayed,
                    [&](hipStream_t gs, int seg) { return launch_fast(g, p, f, out, gs, seg); });
    if (s != NLP_OK) return s;
    // NLP_DIRECT_LAUNCH=1 (stamp-timed sort path): kernels launched one by one,
    // no graph and no events -- the GPU starts after the first launch and the
    // later launches overlap the running kernels
    const bool direct_nomark = stamps && (g->direct_launch || async_direct);
    if (!replayed) {
      if (async && !direct_nomark) return NLP_ERR_DEVICE;  // unreachable: async calls follow a replayed one
      s = sorted ? launch_sp(g, p, sp, out, st, direct_nomark ? -2 : -1) : launch_fast(g, p, f, out, st, -1);
      if (s != NLP_OK) return s;
    }
    if (async) {  // no wait: the fused path's descriptors clean themselves when the call succeeds
      if (sorted && sp.fused) g->ord_clean = sp.arena;
      *handled = true;
      return NLP_OK;
    }
    hipEvent_t* E = (replayed && g->last_single) ? g->gev : g->ev;
    if (hprof) t2 = now_us();
    if ((gseq && stamps && replayed && g->last_single) || direct_nomark) TRY(wait_stream(st));
    else if (stamps && replayed && g->last_single && g->end_mode != 0) TRY(wait_event(g->gev_end));
    else TRY(wait_event(E[2]));
    if (hprof) t3 = now_us();
    const uint64_t* h = sorted ? (const uint64_t*)g->host_ctr : g->host_small;
    if (debug_on())
      fprintf(stderr, "nlp: fast attempt %d range [%llu,%llu) msd %d passes %d split %d capW %llu W %llu C %llu "
              "flags %llx replayed %d\n", attempt, (unsigned long long)p.ua, (unsigned long long)p.ub, (int)msd,
              sorted ? sp.msd_passes : 0, sorted ? (int)sp.split : 0, (unsigned long long)g->capW,
              (unsigned long long)h[C_W], (unsigned long long)h[C_C], (unsigned long long)h[C_FLAGS], (int)replayed);
    if (h[C_FLAGS] >> 32) {  // look-back timeout
      if (debug_on())
        fprintf(stderr, "nlp: look-back timeout, flags %llx W %llu C %llu msd %d passes %d\n",
                (unsigned long long)h[C_FLAGS], (unsigned long long)h[C_W], (unsigned long long)h[C_C], (int)msd,
                msd_passes);
      return NLP_ERR_DEVICE;
    }
    if (h[C_FLAGS] & F_OVERFLOW) {
      const uint64_t W = h[C_W];
      if (!sorted) {  // the grouping did not run: its counters are dirty
        TRY(hipMemsetAsync(g->ws.p[B_UCNT], 0, g->span * 4, st));
        TRY(hipMemsetAsync(g->ws.p[B_IEP], 0, g->span * 4, st));
      }
      if (W > g->wedge_budget) return NLP_OK;
      g->capW = std::max(g->capW, W + W / 4 + 1024);
      continue;
    }
    if (sorted && msd && (h[C_FLAGS] & F_TOOBIG) && h[C_W] <= g->wedge_budget) {
      if (sp.split && sp.msd_passes == 1) msd_passes = 2;
      else msd = false;
      continue;
    }
    if (sorted && sp.counted && (h[C_FLAGS] & F_CPASS)) {  // more than CP_MAXT candidate tiles: look-back passes
      g->cp_off_w = est_w;
      continue;
    }
    if (sorted && sp.small && (h[C_FLAGS] & F_SMALL)) {  // more than SO_MAX candidates: the counted passes
      g->small_off_w = std::max(est_w, 1.0);
      continue;
    }
    if (sorted && sp.fused && !(h[C_FLAGS] >> 32)) g->ord_clean = sp.arena;  // self-cleaned (or never written)
    g->last_wedges = h[C_W];
    if (sorted && !(h[C_FLAGS] & F_TOOBIG)) {
      g->last_ok_w = est_w;
      g->last_ok_msd = msd;
      g->last_ok_passes = msd_passes;
    }
    if ((h[C_FLAGS] & F_TOOBIG) || h[C_W] > g->wedge_budget) return NLP_OK;
    *out_count = h[C_OUT_N];
    // the same call may be replayed without a wait next time (nlp_predict_device_async)
    g->async_ok = sorted && attempt == 0 && ((replayed && g->last_single && stamps) || direct_nomark);
    if (g->async_ok) {
      async_key_of(p, g->async_key);
      g->async_out = out;
    }
    if (result) *result = out;
    if (t) {
      float a = 0, b = 0, hot = 0;
      const bool stamped = stamps && ((replayed && g->last_single) || direct_nomark);
      if (stamped) {
        // the kernels' own stamps -- no event nodes in the graph
        stamp_times(h, &a, &b, &hot);
      } else {
        const hipEvent_t split = sorted ? E[4] : E[1];  // sort grouping: event 4 ends the scoring kernel
        TRY(hipEventElapsedTime(&a, E[0], split));
        TRY(hipEventElapsedTime(&b, split, E[2]));
        TRY(hipEventElapsedTime(&hot, E[3], E[4]));
      }
      const uint64_t nU = std::min(p.ub, g->span) - std::min(p.ua, g->span);
      t->score_ms = a;
      t->select_ms = b;
      t->total_ms = a + b;
      t->wedges = h[C_W];
      t->candidates = h[C_C];
      t->nan_candidates = h[C_NAN];
      t->path = 1;
      t->chunks = 0;
      t->hot_ms = hot;
      t->graph_replay = replayed ? 1u : 0u;
      if (sorted) {
        const int s_runs = 4 + (sp.msd ? sp.msd_passes : sp.passes) + (sp.split ? 1 : 0);
        const int hs = g->hot_stage < 0 ? sp_hot_default(sp) : std::min(std::max(g->hot_stage, 1), s_runs);
        t->hot_bytes = sp_stage_bytes(g, sp, hs, h, p.H);
        t->call_bytes = 0;
        for (int s2 = 1; s2 <= s_runs; ++s2) t->call_bytes += sp_stage_bytes(g, sp, s2, h, p.H);
        t->call_bytes += 12 * h[C_C] + 12 * h[C_OUT_N];  // ordering: candidate columns in, links out
        t->hot_kernel = (sp.fused && hs == s_runs - 1) ? 9u
                        : hs == s_runs ? (sp.split ? 7u : sp.msd ? 1u : 2u)
                        : (sp.split && hs == s_runs - 1) ? (sp.msd_passes == 1 && g->group_sort != 1 && !sp.direct ? 1u : 8u)
                        : hs == 1 ? 4u : hs == 2 ? (sp.fused ? 10u : 5u) : hs >= 4 ? 6u : 0u;
        if (stamped && sp.fused && g->hot_stage < 0) {
          // the fused call's three stamped spans -- k_sp_exbucket (its entry to grouprun's), k_sp_grouprun,
          // and the one-launch ordering k_sp_order_rank (grouprun's end to the last tile) -- and the roofline
          // reports the LONGEST of them, with its own algorithmic bytes
          const uint64_t* tsv = h + NCTR;
          const uint64_t first = ~tsv[TS_FIRST], hin = ~tsv[TS_HOT_IN], hout = tsv[TS_HOT_OUT], end = tsv[TS_END];
          const float exb = hin > first && tsv[TS_FIRST] ? (float)((hin - first) * 1e-5) : 0.0f;
          const float ord = sp.small && end > hout && hout ? (float)((end - hout) * 1e-5) : 0.0f;
          if (exb > t->hot_ms && exb >= ord) {
            t->hot_ms = exb;
            t->hot_bytes = sp_stage_bytes(g, sp, 2, h, p.H);
            t->hot_kernel = 10u;
          } else if (ord > t->hot_ms) {
            t->hot_ms = ord;
            t->hot_bytes = 28 * h[C_C] + 12 * h[C_OUT_N];  // keys + candidate columns in, links out
            t->hot_kernel = 12u;
          }
        }
      } else {
        // k_group_tiles: bucket counts, records, flags, runs
        t->hot_bytes = 4 * nU + 8 * h[C_W] + 4 * h[C_W] + 12 * h[C_C];
        t->hot_kernel = 3;
      }
    }
    if (hprof) {
      hp.prep += t1 - t0;
      hp.launch += t2 - t1;
      hp.wait += t3 - t2;
      hp.post += now_us() - t3;
      constexpr int every = 1000;
      if (++hp.n == every) {
        fprintf(stderr, "nlp host us/call: prepare %.1f launch %.1f wait %.1f post %.1f (replayed %d)\n",
                hp.prep / every, hp.launch / every, hp.wait / every, hp.post / every, (int)replayed);
        hp = HostProf();
      }
    }
    if (g->d_stamp && !g->stamp_path.empty()) {  // diagnostics: append this call's stamps
      std::vector<uint64_t> hs(8 * 65536);
      TRY(hipMemcpy(hs.data(), g->d_stamp, hs.size() * 8, hipMemcpyDeviceToHost));
      if (FILE* fp = fopen(g->stamp_path.c_str(), "ab")) {
        fwrite(hs.data(), 8, hs.size(), fp);
        fclose(fp);
      }
    }
    if (g->async_ok && t) g->async_tmpl = *t;
    *handled = true;
    return NLP_OK;
  }
  return NLP_OK;
}

nlp_status predict_once(nlp_graph* g, const Params& p, EdgeOut* d_out, uint64_t* out_count, nlp_timing* t,
                        hipStream_t st, EdgeOut** result);

// A call that runs out of HBM is retried once with the per-call workspace
// released first: the buffers only grow (a long-lived handle keeps what its
// largest earlier call needed -- a C4 AA H = 32 call then left too little for
// the next Jaccard H = 32 call).
nlp_status predict_impl(nlp_graph* g, const Params& p, EdgeOut* d_out, uint64_t* out_count, nlp_timing* t,
                        hipStream_t st, EdgeOut** result) {
  nlp_status s = predict_once(g, p, d_out, out_count, t, st, result);
  if (s != NLP_ERR_NOMEM) return s;
  (void)hipGetLastError();
  if (hipStreamSynchronize(st) != hipSuccess) return NLP_ERR_DEVICE;
  g->ws.release();
  g->ord_clean = nullptr;     // state keyed by workspace addresses: a new buffer may reuse one
  g->es_desc_bytes = 0;
  g->es_desc_ptr = nullptr;
  g->async_ok = false;
  if (g->hp_scratch) {
    (void)hipFree(g->hp_scratch);
    g->hp_scratch = nullptr;
  }
  return predict_once(g, p, d_out, out_count, t, st, result);
}

nlp_status predict_once(nlp_graph* g, const Params& p, EdgeOut* d_out, uint64_t* out_count, nlp_timing* t,
                        hipStream_t st, EdgeOut** result) {
  // path 3 (hash accumulation) once the wedge count is large: bounded memory,
  // no wedge materialisation (NLP_HASH=1 forces it, NLP_HASH=0 disables it).
  // Adamic-Adar / Resource-Allocation too: their ordered sums are the row
  // kernels' ordered accumulation and the hub pass's sort-mode items
  // (NLP_HASH_AA=0 keeps them on the sort paths, as before round 3)
  const bool custom = p.metric == M_AA || p.metric == M_RA;
  if (t) memset(t, 0, sizeof(*t));  // every path fills its own fields
  // a synchronous call may change what an asynchronous replay would rebuild
  // (capacities, the grouping memo, the range index): only the call that ends
  // eligible below may be replayed
  g->async_ok = false;
  const bool use_hash = !g->force_radix && p.max_edges > 0 &&
                        (g->hash_mode > 0 ||
                         (g->hash_mode == 0 && (!custom || g->hp_aa) && hp_estimate(g, p) > (double)g->hp_min_wedges));
  if (!use_hash && (p.H > 0 || g->sort_grouping) && !g->force_radix && p.max_edges > 0 && p.ua < p.ub && p.ua < g->span) {
    bool handled = false;
    nlp_status s = predict_fast(g, p, d_out, out_count, t, st, result, &handled);
    if (s != NLP_OK || handled) return s;
  }
  Cands C;
  C.metric = p.metric;
  uint32_t path = 0, chunks = 0;
  bool have_nan = false;
  TRY(hipEventRecord(g->ev[0], st));
  if (p.max_edges > 0 && p.ua < p.ub && p.ua < g->span) {
    bool done = false;
    if (use_hash) {
      nlp_status s = run_path3(g, p, C, &chunks, st);
      if (s != NLP_OK) return s;
      done = true;
      path = 4;
      have_nan = true;
    }
    if (!done && p.H > 0 && !g->force_radix) {
      uint64_t fl = 0;
      bool over = false;
      nlp_status s = run_path1_v1(g, p, C, &fl, &over, st);
      if (s != NLP_OK) return s;
      if (!over && !(fl & F_TOOBIG)) {
        done = true;
        path = 1;
        have_nan = true;
      } else {
        C = Cands();
      }
    }
    if (!done && p.H > 0) {  // intermediate-centric with the radix grouping (any bucket size)
      bool fits = false;
      nlp_status s = run_path1(g, p, C, &fits, st);
      if (s != NLP_OK) return s;
      if (fits) { done = true; path = 3; } else C = Cands();
    }
    if (!done) {
      nlp_status s = run_path2(g, p, C, &chunks, st);
      if (s != NLP_OK) return s;
      path = 2;
    }
  }
  TRY(hipEventRecord(g->ev[1], st));
  if (!have_nan) {
    nlp_status s = count_nan(g, C, st);
    if (s != NLP_OK) return s;
  }
  uint64_t total = C.total, nan = C.nan;
  // path 4 may leave its last prune to the order (C.keep: hp_final_order)
  nlp_status s = C.keep ? NLP_OK : prune_to(g, C, p.max_edges, st);
  if (s != NLP_OK) return s;
  if (!d_out) TRY(wsget(g->ws, B_EDGES, std::max<uint64_t>(C.keep ? C.keep : C.n, 1), &d_out));
  s = path == 4 ? hp_final_order(g, C, d_out, st) : order_v1(g, C, d_out, st);
  if (s != NLP_OK) return s;
  TRY(hipEventRecord(g->ev[2], st));
  TRY(hipEventSynchronize(g->ev[2]));
  *out_count = C.n;
  if (result) *result = d_out;
  if (t) {
    float a = 0, b = 0;
    TRY(hipEventElapsedTime(&a, g->ev[0], g->ev[1]));
    TRY(hipEventElapsedTime(&b, g->ev[1], g->ev[2]));
    t->score_ms = a;
    t->select_ms = b;
    t->total_ms = a + b;
    t->wedges = C.wedges;
    t->candidates = total;
    t->nan_candidates = nan;
    t->path = path;
    t->chunks = chunks;
    t->hot_ms = (float)C.hot_ms;
    t->hot_bytes = C.hot_bytes;
    t->hot_kernel = C.hot_launches ? 11u : 0u;
    t->call_bytes = path == 4 ? C.call_bytes : 0;
    t->order_route = path == 4 ? C.route : 0u;
    t->graph_replay = 0;
  }
  return NLP_OK;
}


// ================================================================ multi-device group
// nlp_graph_create_multi: a handle over P logical partitions of the source
// range, partition p on device devices[p] (a device may hold several).  Each
// distinct device keeps one full replica of the graph (second-hop lists are
// arbitrary); partitions run concurrently across devices, one
// host thread per device, and sequentially on a device.

// Partition bounds balanced by the wedge work of hub threshold H, computed
// once per H on the first device (k_hp_work_edges, k_part_weight, a scan and
// P - 1 binary searches).
nlp_status group_bounds(nlp_graph* g, uint32_t H) {
  if (g->part_H == (int64_t)H) return NLP_OK;
  nlp_graph* m = g->members[0];
  TRY(hipSetDevice(m->device));
  hipStream_t st = m->stream;
  const uint64_t S = m->span, M = m->nnz;
  const uint32_t P = (uint32_t)g->part_member.size();
  std::vector<uint64_t> b(P + 1, 0);
  b[P] = S;
  if (P > 1) {
    unsigned long long* wu = nullptr;
    uint64_t *w = nullptr, *pre = nullptr, *scr = nullptr, *bd = nullptr;
    hipError_t e = hipMalloc(&wu, (S + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&w, (S + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&pre, (S + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&scr, (scan_scratch_words(S) + 16) * 8);
    if (e == hipSuccess) e = hipMalloc(&bd, P * 8);
    if (e == hipSuccess) e = hipMemsetAsync(wu, 0, (S + 1) * 8, st);
    if (e == hipSuccess && M) {
      hipLaunchKernelGGL(k_hp_work_edges, dim3((unsigned)std::min<uint64_t>((M + NT * HP_WR - 1) / (NT * HP_WR) + 1, 8192)),
                         dim3(NT), 0, st, view_of(m, M_CN), H, (uint64_t)0, S, (uint64_t)0, M,
                         (const uint32_t*)m->tile_row, wu);
      e = hipGetLastError();
    }
    if (e == hipSuccess) {
      LAUNCH(k_part_weight, S, st, (const unsigned long long*)wu, S, w);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = scan_excl_u64<uint64_t>(w, S, pre, pre + S, scr, st);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_split_points, dim3(1), dim3(std::max<uint32_t>(P, 64)), 0, st, (const uint64_t*)pre, S, P, bd);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(b.data() + 1, bd, (P - 1) * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    for (void* x : {(void*)wu, (void*)w, (void*)pre, (void*)scr, (void*)bd})
      if (x) (void)hipFree(x);
    TRY(e);
    for (uint32_t r = 1; r <= P; ++r) b[r] = std::min(std::max(b[r], b[r - 1]), S);
  }
  g->part_bounds = b;
  g->part_H = H;
  return NLP_OK;
}

// A device buffer of the group, on member `mi`'s device, grown to `n` entries.
template <typename T>
hipError_t group_buf(nlp_graph* g, int mi, T** buf, uint64_t* cap, uint64_t n) {
  if (*cap >= n && *buf) return hipSuccess;
  NLP_HIP(hipSetDevice(g->members[mi]->device));
  if (*buf) NLP_HIP(hipFree(*buf));
  *buf = nullptr;
  *cap = 0;
  NLP_HIP(hipMalloc(buf, std::max<uint64_t>(n, 1) * sizeof(T)));
  *cap = n;
  return hipSuccess;
}

// Key histogram (level 0: key >> 16; level 1: key & 0xffff inside bin `hi`) of
// every partition's list -> per partition 65536 counts.
nlp_status group_hist(nlp_graph* g, const std::vector<uint64_t>& n, int level, uint32_t hi,
                      std::vector<std::vector<uint64_t>>& cnt) {
  const size_t P = g->part_member.size();
  std::vector<std::vector<uint64_t>> fl(P, std::vector<uint64_t>(2 * 65536));
  for (size_t q = 0; q < P; ++q) {
    nlp_graph* m = g->members[g->part_member[q]];
    TRY(hipSetDevice(m->device));
    if (!g->part_hist[q]) TRY(hipMalloc(&g->part_hist[q], 2 * 65536 * 8));
    TRY(hipMemsetAsync(g->part_hist[q], 0, 2 * 65536 * 8, m->stream));
    if (n[q])
      LAUNCH(k_sorted_hist, n[q], m->stream, (const EdgeOut*)(g->part_buf[q] + 1), n[q], level, hi, g->part_hist[q],
             g->part_hist[q] + 65536);
    TRY(hipGetLastError());
    TRY(hipMemcpyAsync(fl[q].data(), g->part_hist[q], 2 * 65536 * 8, hipMemcpyDeviceToHost, m->stream));
  }
  cnt.assign(P, std::vector<uint64_t>(65536, 0));
  for (size_t q = 0; q < P; ++q) {
    nlp_graph* m = g->members[g->part_member[q]];
    TRY(hipSetDevice(m->device));
    TRY(hipStreamSynchronize(m->stream));
    for (int b = 0; b < 65536; ++b)
      if (fl[q][b]) cnt[q][b] = fl[q][65536 + b] - fl[q][b] + 1;
  }
  return NLP_OK;
}

// predictLinks<Metric>Omp over the group: every partition's canonical top-k,
// then the histogram-first selection and one merge on the first device.
// d_out (on devices[0]) may be NULL: the result then stays in group_out.
nlp_status predict_group(nlp_graph* g, const Params& p, EdgeOut* d_out, uint64_t* out_count, nlp_timing* t,
                         EdgeOut** result) {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t P = g->part_member.size();
  nlp_graph* m0 = g->members[0];
  *out_count = 0;
  nlp_status s = group_bounds(g, p.H);
  if (s != NLP_OK) return s;
  std::vector<uint64_t> n(P, 0);
  std::vector<nlp_timing> tp(P);
  std::vector<nlp_status> sm(g->members.size(), NLP_OK);
  const bool bounded = p.max_edges != UINT64_MAX;
  // 1. the partitions' lists (entries 1..n of part_buf), one host thread per device
  auto run_member = [&](size_t mi) {
    nlp_graph* m = g->members[mi];
    if (hipSetDevice(m->device) != hipSuccess) { sm[mi] = NLP_ERR_DEVICE; return; }
    for (size_t q = 0; q < P; ++q) {
      if ((size_t)g->part_member[q] != mi) continue;
      Params pq = p;
      pq.ua = std::max(p.ua, g->part_bounds[q]);
      pq.ub = std::min(p.ub, g->part_bounds[q + 1]);
      memset(&tp[q], 0, sizeof(nlp_timing));
      if (pq.ua >= pq.ub || p.max_edges == 0) continue;
      nlp_status r;
      if (bounded) {
        if (group_buf(g, (int)mi, &g->part_buf[q], &g->part_cap[q], p.max_edges + 1) != hipSuccess) {
          sm[mi] = NLP_ERR_NOMEM;
          return;
        }
        r = predict_impl(m, pq, g->part_buf[q] + 1, &n[q], &tp[q], m->stream, nullptr);
      } else {  // all candidates: kept in the member's workspace, then copied behind the header slot
        EdgeOut* res = nullptr;
        r = predict_impl(m, pq, nullptr, &n[q], &tp[q], m->stream, &res);
        if (r == NLP_OK && group_buf(g, (int)mi, &g->part_buf[q], &g->part_cap[q], n[q] + 1) != hipSuccess)
          r = NLP_ERR_NOMEM;
        if (r == NLP_OK && n[q] &&
            hipMemcpyAsync(g->part_buf[q] + 1, res, n[q] * sizeof(EdgeOut), hipMemcpyDeviceToDevice, m->stream) !=
                hipSuccess)
          r = NLP_ERR_DEVICE;
      }
      if (r == NLP_OK && hipStreamSynchronize(m->stream) != hipSuccess) r = NLP_ERR_DEVICE;
      if (r != NLP_OK) { sm[mi] = r; return; }
    }
  };
  if (g->members.size() == 1) {
    run_member(0);
  } else {
    std::vector<std::thread> th;
    for (size_t mi = 0; mi < g->members.size(); ++mi) th.emplace_back(run_member, mi);
    for (auto& x : th) x.join();
  }
  for (nlp_status r : sm)
    if (r != NLP_OK) return r;
  const auto t1 = std::chrono::steady_clock::now();
  // 2. histogram-first selection: the k-th key, every partition's share
  uint64_t total = 0;
  for (uint64_t x : n) total += x;
  const uint64_t take = std::min(p.max_edges, total);
  std::vector<uint64_t> share(P, 0);
  if (take == total) {
    share = n;
  } else if (take > 0) {
    std::vector<std::vector<uint64_t>> hc, lc;
    s = group_hist(g, n, 0, 0, hc);
    if (s != NLP_OK) return s;
    uint64_t acc = 0;
    int b = 65535;
    for (; b >= 0; --b) {
      uint64_t h = 0;
      for (size_t q = 0; q < P; ++q) h += hc[q][b];
      if (acc + h >= take) break;
      acc += h;
    }
    s = group_hist(g, n, 1, (uint32_t)b, lc);
    if (s != NLP_OK) return s;
    int l = 65535;
    for (; l >= 0; --l) {
      uint64_t h = 0;
      for (size_t q = 0; q < P; ++q) h += lc[q][l];
      if (acc + h >= take) break;
      acc += h;
    }
    uint64_t quota = take - acc;  // ties at the k-th key, handed out in partition (= u) order
    for (size_t q = 0; q < P; ++q) {
      uint64_t above = 0;
      for (int x = b + 1; x < 65536; ++x) above += hc[q][x];
      for (int x = l + 1; x < 65536; ++x) above += lc[q][x];
      const uint64_t tq = std::min(lc[q][l], quota);
      quota -= tq;
      share[q] = above + tq;
    }
  }
  // 3. headers, then the shares to the first device (peer copies over xGMI
  //    between devices, device copies within one)
  uint64_t stride = 1;
  for (uint64_t x : share) stride = std::max(stride, x + 1);
  std::vector<uint32_t> hdr(3 * P);
  for (size_t q = 0; q < P; ++q) {
    hdr[3 * q] = (uint32_t)(share[q] & 0xffffffffu);
    hdr[3 * q + 1] = (uint32_t)(share[q] >> 32);
    hdr[3 * q + 2] = NLP_BLOCK_MAGIC;
  }
  TRY(group_buf(g, 0, &g->gather_buf, &g->gather_cap, stride * P));
  TRY(hipSetDevice(m0->device));
  for (size_t q = 0; q < P; ++q) {
    nlp_graph* m = g->members[g->part_member[q]];
    EdgeOut* dst = g->gather_buf + q * stride;
    TRY(hipMemcpyAsync(dst, &hdr[3 * q], sizeof(EdgeOut), hipMemcpyHostToDevice, m0->stream));
    if (!share[q]) continue;
    if (m->device == m0->device)
      TRY(hipMemcpyAsync(dst + 1, g->part_buf[q] + 1, share[q] * sizeof(EdgeOut), hipMemcpyDeviceToDevice,
                         m0->stream));
    else
      TRY(hipMemcpyPeerAsync(dst + 1, m0->device, g->part_buf[q] + 1, m->device, share[q] * sizeof(EdgeOut),
                             m0->stream));
  }
  // 4. one merge (select.hpp) in canonical order: score desc, then partition = u order
  EdgeOut* out = d_out;
  if (!out) {
    TRY(group_buf(g, 0, &g->group_out, &g->group_out_cap, std::max<uint64_t>(take, 1)));
    TRY(hipSetDevice(m0->device));
    out = g->group_out;
  }
  uint64_t cnt = 0;
  if (take > 0) {
    s = nlp_merge_blocks_device(m0, (const nlp_edge*)g->gather_buf, stride, (uint32_t)P, take, (nlp_edge*)out, &cnt,
                                m0->stream);
    if (s != NLP_OK) return s;
  }
  TRY(hipStreamSynchronize(m0->stream));
  *out_count = cnt;
  if (result) *result = out;
  if (t) {
    memset(t, 0, sizeof(*t));
    const double tot = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const double sc = std::chrono::duration<double, std::milli>(t1 - t0).count();
    t->score_ms = (float)sc;
    t->select_ms = (float)(tot - sc);
    t->total_ms = (float)tot;
    for (size_t q = 0; q < P; ++q) {
      t->wedges += tp[q].wedges;
      t->candidates += tp[q].candidates;
      t->nan_candidates += tp[q].nan_candidates;
      t->path = std::max(t->path, tp[q].path);
      t->chunks += tp[q].chunks;
    }
  }
  return NLP_OK;
}


// ================================================================ N1 / N2 on the device
// (csrc/ingest.hpp; SURVEY §8(f): the reference's ingest and deletion batch)

struct DevTmp {  // device scratch of one call, freed on every exit
  std::vector<void*> p;
  ~DevTmp() {
    for (void* x : p)
      if (x) (void)hipFree(x);
  }
  template <typename T>
  hipError_t get(T** out, uint64_t n) {
    void* x = nullptr;
    hipError_t e = hipMalloc(&x, std::max<uint64_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) p.push_back(x);
    *out = (T*)x;
    return e;
  }
};

// stable LSD sort of u64 keys on the given byte shifts; the sorted keys end in *k
hipError_t sort_u64_keys(uint64_t** k, uint64_t** k2, uint64_t n, const int* shifts, int np, DevTmp& tmp,
                         hipStream_t st) {
  if (n <= 1) return hipSuccess;
  const uint64_t nb = rs_blocks(n);
  uint32_t* hist;
  uint64_t *hoff, *scan;
  NLP_HIP(tmp.get(&hist, (uint64_t)RS_BINS * nb));
  NLP_HIP(tmp.get(&hoff, (uint64_t)RS_BINS * nb));
  NLP_HIP(tmp.get(&scan, scan_scratch_words((uint64_t)RS_BINS * nb) + 16));
  SortScratch sc{hist, hoff, scan, nb};
  int which = 0;
  NLP_HIP(sort_pairs_u64(*k, nullptr, *k2, nullptr, n, shifts, np, sc, &which, st));
  if (which) std::swap(*k, *k2);
  return hipSuccess;
}

// the byte shifts covering a u64 key whose high word holds hbits bits above bit `hi`
// and whose low part holds lbits bits
int key_shifts(int lbits, int hi, int hbits, int* shifts) {
  int np = 0;
  for (int b = 0; b < lbits; b += 8) shifts[np++] = b;
  for (int b = hi; b < hi + hbits; b += 8) shifts[np++] = b;
  return np;
}

// sorted unique keys: compact in place into *out (count in *n_out)
nlp_status unique_keys(const uint64_t* k, uint64_t n, uint64_t* out, uint64_t* n_out, DevTmp& tmp, hipStream_t st) {
  uint8_t* flag;
  uint64_t *pos, *scan;
  TRY(tmp.get(&flag, n));
  TRY(tmp.get(&pos, n + 1));
  TRY(tmp.get(&scan, scan_scratch_words(n) + 16));
  LAUNCH(k_in_first, n, st, k, n, flag);
  TRY(hipGetLastError());
  TRY(scan_excl_u64<uint8_t>(flag, n, pos, pos + n, scan, st));
  LAUNCH(k_in_compact<uint64_t>, n, st, k, (const uint8_t*)flag, (const uint64_t*)pos, n, out);
  TRY(hipGetLastError());
  TRY(hipMemcpyAsync(n_out, pos + n, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  return NLP_OK;
}

}  // namespace

extern "C" {

nlp_status nlp_ingest_device(const uint32_t* d_src, const uint32_t* d_dst, uint64_t m, uint64_t n,
                             int symmetric_input, uint64_t* d_off, uint32_t* d_keys, uint64_t keys_cap,
                             uint64_t* nnz, int device, void* stream) {
  if (!nnz || !d_off || (m && (!d_src || !d_dst)) || n >= (1ull << 31)) return NLP_ERR_INVALID;
  *nnz = 0;
  nlp_status s = check_device(device);
  if (s != NLP_OK) return s;
  TRY(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  const uint64_t span = n + 1;
  DevTmp tmp;
  const int vb = std::max(1, bits_for(n));
  uint64_t ne = 0;
  uint64_t *e = nullptr, *e2 = nullptr;
  if (m) {  // readMtxOmpW: every row sorted and unique
    TRY(tmp.get(&e, m));
    TRY(tmp.get(&e2, m));
    uint32_t* bad;
    TRY(tmp.get(&bad, 1));
    TRY(hipMemsetAsync(bad, 0, 4, st));
    LAUNCH(k_in_pairs, m, st, d_src, d_dst, m, n, e, bad);
    TRY(hipGetLastError());
    uint32_t hbad = 0;
    TRY(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    if (hbad) return NLP_ERR_INVALID;  // an id above n: nothing is written
    int shifts[16];
    const int np = key_shifts(vb, 32, vb, shifts);
    TRY(sort_u64_keys(&e, &e2, m, shifts, np, tmp, st));
    s = unique_keys(e, m, e2, &ne, tmp, st);
    if (s != NLP_OK) return s;
    std::swap(e, e2);  // the distinct pairs, sorted
  }
  // the union entries (row << 33 | key << 1 | tag), sorted
  const uint64_t nent = symmetric_input ? ne : 2 * ne;
  uint64_t *ent = nullptr, *ent2 = nullptr;
  TRY(tmp.get(&ent, nent));
  if (ne && symmetric_input) {  // the rows as read: tag-0 entries, already in (row, key) order
    LAUNCH(k_in_row_entries, ne, st, (const uint64_t*)e, ne, ent);
    TRY(hipGetLastError());
  } else if (ne) {  // symmetrizeOmp's entries: both directions, sorted by (row, key, tag)
    TRY(tmp.get(&ent2, nent));
    LAUNCH(k_in_sym_entries, ne, st, (const uint64_t*)e, ne, ent);
    TRY(hipGetLastError());
    int shifts[16];
    const int np = key_shifts(std::min(64, 1 + vb), 33, vb, shifts);
    TRY(sort_u64_keys(&ent, &ent2, nent, shifts, np, tmp, st));
  }
  // t_v (symmetrize) and the keep flags of the union and of removeSelfLoops
  uint32_t* t;
  uint8_t* keep;
  uint64_t *pos, *scan;
  TRY(tmp.get(&t, span));
  TRY(tmp.get(&keep, nent));
  TRY(tmp.get(&pos, nent + 1));
  TRY(tmp.get(&scan, scan_scratch_words(nent) + 16));
  TRY(hipMemsetAsync(t, 0xff, span * 4, st));
  if (nent) {
    if (!symmetric_input) LAUNCH(k_in_first_absent, nent, st, (const uint64_t*)ent, nent, t);
    LAUNCH(k_in_keep, nent, st, (const uint64_t*)ent, nent, (const uint32_t*)t, symmetric_input ? 0 : 1, keep);
    TRY(hipGetLastError());
  }
  TRY(scan_excl_u64<uint8_t>(keep, nent, pos, pos + nent, scan, st));
  uint64_t total = 0;
  TRY(hipMemcpyAsync(&total, pos + nent, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  *nnz = total;
  if (total > keys_cap || (total && !d_keys)) return NLP_ERR_CAPACITY;
  if (nent) {
    LAUNCH(k_in_scatter_keys, nent, st, (const uint64_t*)ent, (const uint8_t*)keep, (const uint64_t*)pos, nent, d_keys);
    TRY(hipGetLastError());
  }
  LAUNCH(k_in_offsets, span + 1, st, (const uint64_t*)ent, nent, (const uint64_t*)pos, span, d_off);
  TRY(hipGetLastError());
  TRY(hipStreamSynchronize(st));
  return NLP_OK;
}

nlp_status nlp_delete_edges_device(const uint64_t* d_off, const uint32_t* d_keys, uint64_t span, uint64_t batch,
                                   uint32_t* rng_state, uint64_t* d_off2, uint32_t* d_keys2, uint64_t* nnz2,
                                   uint32_t* d_del_u, uint32_t* d_del_v, uint64_t* ndel, int device, void* stream) {
  if (!d_off || !rng_state || !d_off2 || !nnz2 || !ndel || span == 0 || span > 0xffffffffull ||
      (batch && (!d_del_u || !d_del_v)))
    return NLP_ERR_INVALID;
  *nnz2 = 0;
  *ndel = 0;
  nlp_status s = check_device(device);
  if (s != NLP_OK) return s;
  TRY(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  std::vector<uint64_t> off(span + 1);
  TRY(hipMemcpyAsync(off.data(), d_off, (span + 1) * 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  const uint64_t M = off[span];
  if (M && !d_keys2) return NLP_ERR_INVALID;
  // generateEdgeDeletions(rnd, y, batch, 1, span - 1, true) (batch.hxx:99-112, 29-58): per deletion up
  // to 5 attempts (retry, _utility.hxx:199-203), u = K(1 + (span - 1) U), then K(U deg u) -- the draws
  std::vector<uint32_t> du, di;
  du.reserve(batch);
  di.reserve(batch);
  nlp::Minstd0 rnd(*rng_state);  // a seed, or a state in [1, 2^31 - 2] (which seeds to itself)
  const size_t i0 = 1, n0 = span - 1;
  for (uint64_t l = 0; l < batch; ++l) {
    for (int attempt = 0; attempt < 5; ++attempt) {
      const uint32_t u = (uint32_t)(i0 + n0 * nlp::canonical01(rnd));
      const uint64_t d = u < span ? off[u + 1] - off[u] : 0;
      if (d == 0) continue;
      du.push_back(u);
      di.push_back((uint32_t)(nlp::canonical01(rnd) * d));
      break;
    }
  }
  *rng_state = rnd.x;
  const uint64_t nd = du.size();
  DevTmp tmp;
  uint64_t nt = 0;
  uint64_t *dk = nullptr, *dk2 = nullptr;
  const int vb = std::max(1, bits_for(span - 1));
  if (nd) {
    uint32_t *ddu, *ddi;
    TRY(tmp.get(&ddu, nd));
    TRY(tmp.get(&ddi, nd));
    TRY(hipMemcpyAsync(ddu, du.data(), nd * 4, hipMemcpyHostToDevice, st));
    TRY(hipMemcpyAsync(ddi, di.data(), nd * 4, hipMemcpyHostToDevice, st));
    TRY(tmp.get(&dk, 2 * nd));
    TRY(tmp.get(&dk2, 2 * nd));
    LAUNCH(k_del_pick, nd, st, (const uint32_t*)ddu, (const uint32_t*)ddi, nd, d_off, d_keys, dk);
    TRY(hipGetLastError());
    // tidyBatchUpdateU (batch.hxx:152-208): keep existing, sort, unique
    int shifts[16];
    const int np = key_shifts(vb, 32, vb, shifts);
    TRY(sort_u64_keys(&dk, &dk2, 2 * nd, shifts, np, tmp, st));
    uint8_t* f;
    uint64_t *pos, *scan;
    TRY(tmp.get(&f, 2 * nd));
    TRY(tmp.get(&pos, 2 * nd + 1));
    TRY(tmp.get(&scan, scan_scratch_words(2 * nd) + 16));
    LAUNCH(k_del_tidy, 2 * nd, st, (const uint64_t*)dk, 2 * nd, d_off, d_keys, span, f);
    TRY(hipGetLastError());
    TRY(scan_excl_u64<uint8_t>(f, 2 * nd, pos, pos + 2 * nd, scan, st));
    LAUNCH(k_in_compact<uint64_t>, 2 * nd, st, (const uint64_t*)dk, (const uint8_t*)f, (const uint64_t*)pos, 2 * nd,
           dk2);
    TRY(hipGetLastError());
    TRY(hipMemcpyAsync(&nt, pos + 2 * nd, 8, hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    std::swap(dk, dk2);
  }
  // applyBatchUpdateOmpU (batch.hxx:239-247): one occurrence per deletion leaves its row
  uint8_t *gone, *keep;
  uint64_t *pos, *scan;
  TRY(tmp.get(&gone, M));
  TRY(tmp.get(&keep, M));
  TRY(tmp.get(&pos, M + 1));
  TRY(tmp.get(&scan, scan_scratch_words(M) + 16));
  TRY(hipMemsetAsync(gone, 0, std::max<uint64_t>(M, 1), st));
  if (nt) LAUNCH(k_del_mark, nt, st, (const uint64_t*)dk, nt, d_off, d_keys, span, gone);
  if (M) LAUNCH(k_del_keepflag, M, st, (const uint8_t*)gone, M, keep);
  TRY(hipGetLastError());
  TRY(scan_excl_u64<uint8_t>(keep, M, pos, pos + M, scan, st));
  if (M) LAUNCH(k_in_compact<uint32_t>, M, st, d_keys, (const uint8_t*)keep, (const uint64_t*)pos, M, d_keys2);
  LAUNCH(k_del_offsets, span + 1, st, d_off, span, (const uint64_t*)pos, d_off2);
  if (nt) LAUNCH(k_del_split, nt, st, (const uint64_t*)dk, nt, d_del_u, d_del_v);
  TRY(hipGetLastError());
  uint64_t m2 = 0;
  TRY(hipMemcpyAsync(&m2, pos + M, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  *nnz2 = m2;
  *ndel = nt;
  return NLP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- device CSR (N1 / N2 for host callers)
struct nlp_dcsr {
  int device = 0;
  uint64_t span = 0, nnz = 0;
  uint64_t* off = nullptr;
  uint32_t* keys = nullptr;
  uint64_t read_size = 0, sym_size = 0;  // the graph after readMtx and after symmetrize (N1 stages)
};

namespace {
void dcsr_free(nlp_dcsr* x) {
  if (!x) return;
  (void)hipSetDevice(x->device);
  if (x->off) (void)hipFree(x->off);
  if (x->keys) (void)hipFree(x->keys);
  delete x;
}
}  // namespace

extern "C" {

nlp_status nlp_dcsr_ingest(const uint32_t* src, const uint32_t* dst, uint64_t m, uint64_t n, int symmetric_input,
                           int device, nlp_dcsr** out) {
  if (!out || (m && (!src || !dst)) || n >= (1ull << 31)) return NLP_ERR_INVALID;
  *out = nullptr;
  nlp_status s = check_device(device);
  if (s != NLP_OK) return s;
  TRY(hipSetDevice(device));
  nlp_dcsr* x = new (std::nothrow) nlp_dcsr();
  if (!x) return NLP_ERR_NOMEM;
  x->device = device;
  x->span = n + 1;
  DevTmp tmp;
  uint32_t *ds = nullptr, *dd = nullptr;
  if (tmp.get(&ds, m) != hipSuccess || tmp.get(&dd, m) != hipSuccess ||
      hipMalloc(&x->off, (n + 2) * 8) != hipSuccess || hipMalloc(&x->keys, std::max<uint64_t>(2 * m, 1) * 4) != hipSuccess) {
    dcsr_free(x);
    return NLP_ERR_NOMEM;
  }
  if (m && (hipMemcpy(ds, src, m * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(dd, dst, m * 4, hipMemcpyHostToDevice) != hipSuccess)) {
    dcsr_free(x);
    return NLP_ERR_DEVICE;
  }
  // the stage sizes main.cxx prints: distinct pairs (readMtx), then + the one
  // self loop per row that removeSelfLoops takes out again
  uint64_t* e;
  uint64_t* cnt;
  if (tmp.get(&e, std::max<uint64_t>(m, 1)) != hipSuccess || tmp.get(&cnt, 2) != hipSuccess) {
    dcsr_free(x);
    return NLP_ERR_NOMEM;
  }
  s = nlp_ingest_device(ds, dd, m, n, symmetric_input, x->off, x->keys, std::max<uint64_t>(2 * m, 1), &x->nnz, device,
                        nullptr);
  if (s != NLP_OK) {
    dcsr_free(x);
    return s;
  }
  if (m) {  // distinct pairs and distinct self loops
    // cnt starts clear (k_in_pairs ORs an out-of-range flag into it; nlp_ingest_device has
    // already rejected such ids), and every launch is checked
    if (hipMemset(cnt, 0, 16) != hipSuccess) {
      dcsr_free(x);
      return NLP_ERR_DEVICE;
    }
    LAUNCH(k_in_pairs, m, nullptr, (const uint32_t*)ds, (const uint32_t*)dd, m, n, e, (uint32_t*)cnt);
    if (hipGetLastError() != hipSuccess) {
      dcsr_free(x);
      return NLP_ERR_DEVICE;
    }
    int shifts[16];
    const int vb = std::max(1, bits_for(n));
    const int np = key_shifts(vb, 32, vb, shifts);
    uint64_t* e2;
    if (tmp.get(&e2, m) != hipSuccess) {
      dcsr_free(x);
      return NLP_ERR_NOMEM;
    }
    if (sort_u64_keys(&e, &e2, m, shifts, np, tmp, nullptr) != hipSuccess ||
        hipMemset(cnt, 0, 16) != hipSuccess) {
      dcsr_free(x);
      return NLP_ERR_DEVICE;
    }
    LAUNCH(k_in_count_distinct, m, nullptr, (const uint64_t*)e, m, (unsigned long long*)cnt);
    uint64_t h[2] = {0, 0};
    if (hipGetLastError() != hipSuccess || hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost) != hipSuccess) {
      dcsr_free(x);
      return NLP_ERR_DEVICE;
    }
    x->read_size = h[0];
    x->sym_size = x->nnz + h[1];
  }
  *out = x;
  return NLP_OK;
}

nlp_status nlp_dcsr_delete_batch(const nlp_dcsr* x, uint64_t batch, uint32_t* rng_state, nlp_dcsr** out,
                                 uint32_t* del_u, uint32_t* del_v, uint64_t del_cap, uint64_t* ndel) {
  if (!x || !out || !rng_state || !ndel) return NLP_ERR_INVALID;
  *out = nullptr;
  *ndel = 0;
  TRY(hipSetDevice(x->device));
  nlp_dcsr* y = new (std::nothrow) nlp_dcsr();
  if (!y) return NLP_ERR_NOMEM;
  y->device = x->device;
  y->span = x->span;
  DevTmp tmp;
  uint32_t *du = nullptr, *dv = nullptr;
  if (hipMalloc(&y->off, (x->span + 1) * 8) != hipSuccess ||
      hipMalloc(&y->keys, std::max<uint64_t>(x->nnz, 1) * 4) != hipSuccess || tmp.get(&du, 2 * batch) != hipSuccess ||
      tmp.get(&dv, 2 * batch) != hipSuccess) {
    dcsr_free(y);
    return NLP_ERR_NOMEM;
  }
  uint64_t nd = 0;
  // the engine state is restored on every error return, so a retry (e.g. with a larger
  // deletion buffer) draws the same batch -- the minstd_rand0 replay N2 parity relies on
  const uint32_t rng0 = *rng_state;
  nlp_status s = nlp_delete_edges_device(x->off, x->keys, x->span, batch, rng_state, y->off, y->keys, &y->nnz, du, dv,
                                         &nd, x->device, nullptr);
  if (s != NLP_OK) {
    *rng_state = rng0;
    dcsr_free(y);
    return s;
  }
  *ndel = nd;
  if ((del_u || del_v) && nd > del_cap) {
    *rng_state = rng0;
    dcsr_free(y);
    return NLP_ERR_CAPACITY;
  }
  if (nd && ((del_u && hipMemcpy(del_u, du, nd * 4, hipMemcpyDeviceToHost) != hipSuccess) ||
             (del_v && hipMemcpy(del_v, dv, nd * 4, hipMemcpyDeviceToHost) != hipSuccess))) {
    *rng_state = rng0;
    dcsr_free(y);
    return NLP_ERR_DEVICE;
  }
  y->read_size = y->sym_size = y->nnz;
  *out = y;
  return NLP_OK;
}

nlp_status nlp_dcsr_info(const nlp_dcsr* x, uint64_t* span, uint64_t* nnz, uint64_t* read_size, uint64_t* sym_size) {
  if (!x) return NLP_ERR_INVALID;
  if (span) *span = x->span;
  if (nnz) *nnz = x->nnz;
  if (read_size) *read_size = x->read_size;
  if (sym_size) *sym_size = x->sym_size;
  return NLP_OK;
}

nlp_status nlp_dcsr_copy(const nlp_dcsr* x, uint64_t* off, uint32_t* keys) {
  if (!x) return NLP_ERR_INVALID;
  TRY(hipSetDevice(x->device));
  if (off) TRY(hipMemcpy(off, x->off, (x->span + 1) * 8, hipMemcpyDeviceToHost));
  if (keys && x->nnz) TRY(hipMemcpy(keys, x->keys, x->nnz * 4, hipMemcpyDeviceToHost));
  return NLP_OK;
}

void nlp_dcsr_destroy(nlp_dcsr* x) { dcsr_free(x); }

}  // extern "C"

namespace {

}  // namespace

// ---------------------------------------------------------------- C-ABI

extern "C" {

nlp_status nlp_graph_create(const uint64_t* offsets, const uint32_t* keys, uint64_t span, int device,
                            nlp_graph** out) {
  if (!out || !offsets || span == 0 || span > 0xffffffffull) return NLP_ERR_INVALID;
  *out = nullptr;
  const uint64_t M = offsets[span];
  if (offsets[0] != 0 || (M && !keys)) return NLP_ERR_INVALID;
  nlp_graph* g;
  nlp_status s = new_graph(device, &g);
  if (s != NLP_OK) return s;
  BuildClock clk(g);
  g->span = span;
  g->nnz = M;
  if (hmalloc(&g->off, (span + 1) * 8) != hipSuccess || hmalloc(&g->keys, std::max<uint64_t>(M, 1) * 4) != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_NOMEM;
  }
  if (hipMemcpyAsync(g->off, offsets, (span + 1) * 8, hipMemcpyHostToDevice, g->stream) != hipSuccess ||
      (M && hipMemcpyAsync(g->keys, keys, M * 4, hipMemcpyHostToDevice, g->stream) != hipSuccess)) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  if (clk.mark("upload") != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  s = finish_graph(g, clk);
  if (s != NLP_OK) { destroy_graph(g); return s; }
  *out = g;
  return NLP_OK;
}

nlp_status nlp_graph_create_dcsr(const nlp_dcsr* x, nlp_graph** out) {
  if (!x || !out) return NLP_ERR_INVALID;
  return nlp_graph_create_device(x->off, x->keys, x->span, x->nnz, x->device, nullptr, out);
}

nlp_status nlp_graph_create_device(const uint64_t* d_offsets, const uint32_t* d_keys, uint64_t span, uint64_t nnz,
                                   int device, void* stream, nlp_graph** out) {
  if (!out || !d_offsets || span == 0 || span > 0xffffffffull || (nnz && !d_keys)) return NLP_ERR_INVALID;
  *out = nullptr;
  nlp_graph* g;
  nlp_status s = new_graph(device, &g);
  if (s != NLP_OK) return s;
  BuildClock clk(g);
  g->span = span;
  g->nnz = nnz;
  hipStream_t ust = (hipStream_t)stream;
  if (hmalloc(&g->off, (span + 1) * 8) != hipSuccess || hmalloc(&g->keys, std::max<uint64_t>(nnz, 1) * 4) != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_NOMEM;
  }
  // inputs may come from any stream: order after `stream`, or after everything
  if ((ust ? hipStreamSynchronize(ust) : hipDeviceSynchronize()) != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  if (hipMemcpyAsync(g->off, d_offsets, (span + 1) * 8, hipMemcpyDeviceToDevice, g->stream) != hipSuccess ||
      (nnz && hipMemcpyAsync(g->keys, d_keys, nnz * 4, hipMemcpyDeviceToDevice, g->stream) != hipSuccess)) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  if (clk.mark("upload") != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  s = finish_graph(g, clk);
  if (s != NLP_OK) { destroy_graph(g); return s; }
  *out = g;
  return NLP_OK;
}

}  // extern "C"

// A replica of `src`'s CSR on `device`, copied device to device (peer copies
// over xGMI between GPUs), then the per-graph build of finish_graph.
static nlp_status graph_create_peer(const nlp_graph* src, int device, nlp_graph** out) {
  *out = nullptr;
  nlp_graph* g;
  nlp_status s = new_graph(device, &g);
  if (s != NLP_OK) return s;
  BuildClock clk(g);
  g->span = src->span;
  g->nnz = src->nnz;
  if (hmalloc(&g->off, (g->span + 1) * 8) != hipSuccess || hmalloc(&g->keys, std::max<uint64_t>(g->nnz, 1) * 4) != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_NOMEM;
  }
  if (hipSetDevice(src->device) != hipSuccess || hipStreamSynchronize(src->stream) != hipSuccess ||
      hipSetDevice(device) != hipSuccess ||
      hipMemcpyPeerAsync(g->off, device, src->off, src->device, (g->span + 1) * 8, g->stream) != hipSuccess ||
      (g->nnz && hipMemcpyPeerAsync(g->keys, device, src->keys, src->device, g->nnz * 4, g->stream) != hipSuccess)) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  if (clk.mark("upload") != hipSuccess) {
    destroy_graph(g);
    return NLP_ERR_DEVICE;
  }
  s = finish_graph(g, clk);
  if (s != NLP_OK) { destroy_graph(g); return s; }
  *out = g;
  return NLP_OK;
}

extern "C" {

nlp_status nlp_graph_create_multi(const uint64_t* offsets, const uint32_t* keys, uint64_t span, const int* devices,
                                  int ndev, nlp_graph** out) {
  if (!out || !offsets || !devices || ndev < 1 || ndev > NLP_MAX_PARTS || span == 0 || span > 0xffffffffull)
    return NLP_ERR_INVALID;
  *out = nullptr;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return NLP_ERR_NODEVICE;
  for (int i = 0; i < ndev; ++i) {
    nlp_status s = check_device(devices[i]);
    if (s != NLP_OK) return s;
  }
  nlp_graph* g = new (std::nothrow) nlp_graph();
  if (!g) return NLP_ERR_NOMEM;
  g->is_group = true;
  g->device = devices[0];
  // distinct devices, in order of first appearance (NLP_MULTI_EACH=1: one
  // member per partition even on a repeated device -- exercises the
  // member-to-member copy on a one-GPU box)
  const char* each = getenv("NLP_MULTI_EACH");
  const bool own = each && atoi(each) > 0;
  std::vector<int> devs;
  for (int i = 0; i < ndev; ++i) {
    int mi = own ? (int)devs.size() : (int)(std::find(devs.begin(), devs.end(), devices[i]) - devs.begin());
    if (mi == (int)devs.size()) devs.push_back(devices[i]);
    g->part_member.push_back(mi);
  }
  for (size_t a = 0; a < devs.size(); ++a)  // peer access (xGMI) for the replica copies and the share copies
    for (size_t b = 0; b < devs.size(); ++b)
      if (devs[a] != devs[b] && hipSetDevice(devs[a]) == hipSuccess) {
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, devs[a], devs[b]) == hipSuccess && can) (void)hipDeviceEnablePeerAccess(devs[b], 0);
        (void)hipGetLastError();
      }
  // the host CSR crosses PCIe once, to the first device; the other replicas
  // are copied device to device from it (xGMI peer copies)
  for (size_t i = 0; i < devs.size(); ++i) {
    nlp_graph* m = nullptr;
    nlp_status s = i == 0 ? nlp_graph_create(offsets, keys, span, devs[0], &m) : graph_create_peer(g->members[0], devs[i], &m);
    if (s != NLP_OK) { destroy_graph(g); return s; }
    g->members.push_back(m);
  }
  g->part_buf.assign(ndev, nullptr);
  g->part_cap.assign(ndev, 0);
  g->part_hist.assign(ndev, nullptr);
  g->span = span;
  g->nnz = g->members[0]->nnz;
  g->maxdeg = g->members[0]->maxdeg;
  g->symmetric = g->members[0]->symmetric;
  g->last_stream = g->members[0]->stream;
  *out = g;
  return NLP_OK;
}

int nlp_device_count(void) {
  int n = 0, c = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  for (int d = 0; d < n; ++d)
    if (check_device(d) == NLP_OK) ++c;
  return c;
}

nlp_status nlp_graph_parts(const nlp_graph* g, int* nparts, uint64_t* bounds) {
  if (!g || !nparts) return NLP_ERR_INVALID;
  *nparts = g->is_group ? (int)g->part_member.size() : 1;
  if (bounds) {
    if (g->is_group && g->part_H >= 0)
      for (size_t i = 0; i < g->part_bounds.size(); ++i) bounds[i] = g->part_bounds[i];
    else if (g->is_group)
      return NLP_ERR_INVALID;  // no prediction yet: the bounds depend on the hub threshold
    else {
      bounds[0] = 0;
      bounds[1] = g->span;
    }
  }
  return NLP_OK;
}

void nlp_graph_destroy(nlp_graph* g) { destroy_graph(g); }

nlp_status nlp_graph_info(const nlp_graph* g, uint64_t* span, uint64_t* nnz, uint32_t* max_degree, int* symmetric) {
  if (!g) return NLP_ERR_INVALID;
  if (span) *span = g->span;
  if (nnz) *nnz = g->nnz;
  if (max_degree) *max_degree = g->maxdeg;
  if (symmetric) *symmetric = g->symmetric ? 1 : 0;
  return NLP_OK;
}

nlp_status nlp_set_hot_stage(nlp_graph* g, int stage) {
  if (!g || g->is_group || g->async_pending) return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess || hipStreamSynchronize(g->stream) != hipSuccess) return NLP_ERR_DEVICE;
  if (stage != g->hot_stage) {  // captured graphs carry the old event placement
    for (auto& c : g->graphs)
      for (auto& x : c.exec)
        if (x) (void)hipGraphExecDestroy(x);
    g->graphs.clear();
    g->async_ok = false;
  }
  g->hot_stage = stage < 0 ? -1 : stage;
  return NLP_OK;
}

nlp_status nlp_graph_build_phases(const nlp_graph* g, uint32_t cap, uint32_t* n, const char** names, double* ms,
                                  double* alloc_ms) {
  if (!g || !n) return NLP_ERR_INVALID;
  const nlp_graph* m = g->is_group ? g->members[0] : g;
  *n = (uint32_t)m->build_phases.size();
  for (uint32_t i = 0; i < *n && i < cap; ++i) {
    if (names) names[i] = m->build_phases[i].first;
    if (ms) ms[i] = m->build_phases[i].second;
  }
  if (alloc_ms) *alloc_ms = m->build_alloc_ms;
  return NLP_OK;
}

nlp_status nlp_predict_device_ex(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, uint32_t max_factor2,
                                 float min_score, uint64_t max_edges, uint64_t u_begin, uint64_t u_end, nlp_edge* d_out,
                                 uint64_t* out_count, nlp_timing* t, void* stream) {
  if (!g || !out_count || (int)metric < 0 || (int)metric > 8 || (max_edges && !d_out)) return NLP_ERR_INVALID;
  if (g->async_pending) return NLP_ERR_INVALID;  // an asynchronous batch is in flight: nlp_sync first
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  if (g->is_group) {  // every partition on its device, the merged result into d_out (on devices[0])
    if ((stream ? hipStreamSynchronize((hipStream_t)stream) : hipDeviceSynchronize()) != hipSuccess)
      return NLP_ERR_DEVICE;
    Params p{(int)metric, hub_max_degree, min_score, max_edges, u_begin, std::min<uint64_t>(u_end, g->span),
             max_factor2};
    nlp_timing tt;
    memset(&tt, 0, sizeof(tt));
    g->last_out = nullptr;
    g->last_n = 0;
    nlp_status s = predict_group(g, p, (EdgeOut*)d_out, out_count, &tt, nullptr);
    if (t) *t = tt;
    if (s == NLP_OK) {
      g->last_out = (const EdgeOut*)d_out;
      g->last_n = *out_count;
      g->last_stream = g->members[0]->stream;
    }
    return s;
  }
  hipStream_t st = stream ? (hipStream_t)stream : g->stream;
  // the graph's own stream does not order after other streams: with no caller
  // stream, wait for all prior device work (inputs/outputs may come from it)
  if (!stream && hipDeviceSynchronize() != hipSuccess) return NLP_ERR_DEVICE;
  Params p{(int)metric, hub_max_degree, min_score, max_edges, u_begin, std::min<uint64_t>(u_end, g->span), max_factor2};
  nlp_timing tt;
  memset(&tt, 0, sizeof(tt));
  g->last_out = nullptr;
  g->last_n = 0;
  nlp_status s = predict_impl(g, p, (EdgeOut*)d_out, out_count, &tt, st, nullptr);
  if (t) *t = tt;
  if (s == NLP_OK) {
    g->last_out = (const EdgeOut*)d_out;
    g->last_n = *out_count;
    g->last_stream = st;
  }
  return s;
}

nlp_status nlp_predict_device(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, float min_score,
                              uint64_t max_edges, uint64_t u_begin, uint64_t u_end, nlp_edge* d_out,
                              uint64_t* out_count, nlp_timing* t, void* stream) {
  return nlp_predict_device_ex(g, metric, hub_max_degree, 0, min_score, max_edges, u_begin, u_end, d_out, out_count,
                               t, stream);
}

nlp_status nlp_predict_device_async(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, uint32_t max_factor2,
                                    float min_score, uint64_t max_edges, uint64_t u_begin, uint64_t u_end,
                                    nlp_edge* d_out, void* stream) {
  if (!g || (int)metric < 0 || (int)metric > 8 || (max_edges && !d_out) || g->is_group) return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  // NULL: the device's default stream (ordered after the caller's default-stream work without a
  // device-wide wait; the synchronous entry points use the handle's own stream and a device sync)
  hipStream_t st = (hipStream_t)stream;
  if (g->async_pending && st != g->async_stream) return NLP_ERR_INVALID;  // one stream per batch
  Params p{(int)metric, hub_max_degree, min_score, max_edges, u_begin, std::min<uint64_t>(u_end, g->span), max_factor2};
  uint64_t key[6];
  async_key_of(p, key);
  g->last_out = nullptr;
  g->last_n = 0;
  if (g->async_ok && g->async_out == (const void*)d_out && memcmp(key, g->async_key, sizeof key) == 0) {
    bool handled = false;
    uint64_t cnt = 0;
    // a batch starts with a clean flag word (a synchronous call's own redos are no failure)
    if (!g->async_pending || g->async_last_sync) TRY(hipMemsetAsync(g->d_sticky, 0, 8, st));
    nlp_status s = predict_fast(g, p, (EdgeOut*)d_out, &cnt, nullptr, st, nullptr, &handled, true);
    if (s != NLP_OK) return s;
    if (handled) {
      ++g->async_pending;
      g->async_last_sync = false;
      g->async_stream = st;
      g->async_last_out = d_out;
      return NLP_OK;
    }
  }
  // not replayable: a synchronous call (after folding in the flags of the batch's replayed calls)
  if (g->async_pending && !g->async_last_sync) {
    uint64_t f = 0;
    TRY(hipStreamSynchronize(st));
    TRY(hipMemcpy(&f, g->d_sticky, 8, hipMemcpyDeviceToHost));
    g->async_fail |= f;
  }
  uint64_t cnt = 0;
  nlp_timing tt;
  memset(&tt, 0, sizeof(tt));
  nlp_status s = predict_impl(g, p, (EdgeOut*)d_out, &cnt, &tt, st, nullptr);
  if (s != NLP_OK) return s;
  ++g->async_pending;
  g->async_last_sync = true;
  g->async_count = cnt;
  g->async_t = tt;
  g->async_stream = st;
  g->async_last_out = d_out;
  return NLP_OK;
}

nlp_status nlp_sync(nlp_graph* g, uint64_t* out_count, nlp_timing* t) {
  if (!g || !out_count || !g->async_pending) return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  const bool last_sync = g->async_last_sync;
  g->async_pending = 0;
  TRY(hipStreamSynchronize(g->async_stream));
  uint64_t f = 0;
  if (!last_sync) {
    TRY(hipMemcpy(&f, g->d_sticky, 8, hipMemcpyDeviceToHost));
    TRY(hipMemset(g->d_sticky, 0, 8));
  }
  f |= g->async_fail;
  g->async_fail = 0;
  if ((f & (F_OVERFLOW | F_TOOBIG | F_CPASS | F_SMALL)) || (f >> 32)) {  // some call of the batch needs a redo
    g->ord_clean = nullptr;
    g->async_ok = false;
    return NLP_ERR_RETRY;
  }
  if (last_sync) {
    *out_count = g->async_count;
    if (t) *t = g->async_t;
  } else {
    const uint64_t* h = (const uint64_t*)g->host_ctr;
    *out_count = h[C_OUT_N];
    if (t) {
      *t = g->async_tmpl;  // path, hot kernel and its bytes: those of the same synchronous call
      stamp_times(h, &t->score_ms, &t->select_ms, &t->hot_ms);
      t->total_ms = t->score_ms + t->select_ms;
      t->wedges = h[C_W];
      t->candidates = h[C_C];
      t->nan_candidates = h[C_NAN];
    }
  }
  g->last_out = (const EdgeOut*)g->async_last_out;
  g->last_n = *out_count;
  g->last_stream = g->async_stream;
  return NLP_OK;
}

nlp_status nlp_predict_ex(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, uint32_t max_factor2,
                          float min_score, uint64_t max_edges, int repeat, nlp_edge* out, uint64_t* out_count,
                          nlp_timing* t) {
  if (!g || !out_count || (int)metric < 0 || (int)metric > 8) return NLP_ERR_INVALID;
  if (g->async_pending) return NLP_ERR_INVALID;  // an asynchronous batch is in flight: nlp_sync first
  if (repeat < 1) repeat = 1;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  hipStream_t st = g->stream;
  Params p{(int)metric, hub_max_degree, min_score, max_edges, 0, g->span, max_factor2};
  // measureDuration(fn, repeat) semantics (_utility.hxx:345-352): the timed
  // work runs `repeat` times and the reported times are averages.
  float score_sum = 0, select_sum = 0;
  nlp_timing last;
  memset(&last, 0, sizeof(last));
  EdgeOut* d_res = nullptr;
  uint64_t n = 0;
  g->last_out = nullptr;
  g->last_n = 0;
  if (g->is_group) st = g->members[0]->stream;
  for (int r = 0; r < repeat; ++r) {
    nlp_status s = g->is_group ? predict_group(g, p, nullptr, &n, &last, &d_res)
                               : predict_impl(g, p, nullptr, &n, &last, st, &d_res);
    if (s == NLP_OK && g->is_group) TRY(hipSetDevice(g->device));
    if (s != NLP_OK) return s;
    score_sum += last.score_ms;
    select_sum += last.select_ms;
  }
  last.score_ms = score_sum / repeat;
  last.select_ms = select_sum / repeat;
  last.total_ms = last.score_ms + last.select_ms;
  if (out && n && g->is_group) {
    const auto c0 = std::chrono::steady_clock::now();
    TRY(hipMemcpyAsync(out, d_res, n * sizeof(EdgeOut), hipMemcpyDeviceToHost, st));
    TRY(hipStreamSynchronize(st));
    last.copy_ms = (float)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
  } else if (out && n) {
    TRY(hipEventRecord(g->ev[0], st));
    TRY(hipMemcpyAsync(out, d_res, n * sizeof(EdgeOut), hipMemcpyDeviceToHost, st));
    TRY(hipEventRecord(g->ev[1], st));
    TRY(hipEventSynchronize(g->ev[1]));
    TRY(hipEventElapsedTime(&last.copy_ms, g->ev[0], g->ev[1]));
  }
  *out_count = n;
  if (t) *t = last;
  g->last_out = d_res;
  g->last_n = n;
  g->last_stream = st;
  return NLP_OK;
}

nlp_status nlp_predict(nlp_graph* g, nlp_metric metric, uint32_t hub_max_degree, float min_score, uint64_t max_edges,
                       int repeat, nlp_edge* out, uint64_t* out_count, nlp_timing* t) {
  return nlp_predict_ex(g, metric, hub_max_degree, 0, min_score, max_edges, repeat, out, out_count, t);
}

nlp_status nlp_copy_last(nlp_graph* g, nlp_edge* out, uint64_t n, uint64_t* copied) {
  if (!g || !copied || (n && !out)) return NLP_ERR_INVALID;
  *copied = 0;
  const uint64_t m = std::min(n, g->last_n);
  if (!m) return NLP_OK;
  if (!g->last_out) return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  TRY(hipMemcpyAsync(out, g->last_out, m * sizeof(EdgeOut), hipMemcpyDeviceToHost, g->last_stream));
  TRY(hipStreamSynchronize(g->last_stream));
  *copied = m;
  return NLP_OK;
}

nlp_status nlp_host_alloc(uint64_t bytes, void** out) {
  if (!out) return NLP_ERR_INVALID;
  *out = nullptr;
  if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    *out = nullptr;
    return NLP_ERR_NOMEM;
  }
  return NLP_OK;
}

void nlp_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

nlp_status nlp_set_truth(nlp_graph* g, const uint32_t* u, const uint32_t* v, uint64_t n) {
  if (g && g->is_group) return nlp_set_truth(g->members[0], u, v, n);
  if (!g || (n && (!u || !v))) return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  std::vector<uint64_t> k(n);
  for (uint64_t i = 0; i < n; ++i) k[i] = ((uint64_t)u[i] << 32) | v[i];
  std::sort(k.begin(), k.end());
  k.erase(std::unique(k.begin(), k.end()), k.end());
  if (g->truth) TRY(hipFree(g->truth));
  g->truth = nullptr;
  g->ntruth = k.size();
  TRY(hipMalloc(&g->truth, std::max<uint64_t>(k.size(), 1) * 8));
  if (!k.empty()) TRY(hipMemcpy(g->truth, k.data(), k.size() * 8, hipMemcpyHostToDevice));
  return NLP_OK;
}

nlp_status nlp_count_common_device(nlp_graph* g, const nlp_edge* d_edges, uint64_t n, uint64_t* common,
                                   void* stream) {
  if (g && g->is_group) return nlp_count_common_device(g->members[0], d_edges, n, common, stream);
  if (!g || !common || (n && !d_edges)) return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  hipStream_t st = stream ? (hipStream_t)stream : g->stream;
  *common = 0;
  if (!n || !g->ntruth) return NLP_OK;
  if (!stream && hipDeviceSynchronize() != hipSuccess) return NLP_ERR_DEVICE;
  unsigned long long* c;
  TRY(wsget(g->ws, B_EVAL, 1, &c));
  TRY(hipMemsetAsync(c, 0, 8, st));
  LAUNCH(k_count_common, n, st, (const EdgeOut*)d_edges, n, (const uint64_t*)g->truth, g->ntruth, c);
  TRY(hipGetLastError());
  TRY(hipMemcpyAsync(&g->host_small[0], c, 8, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  *common = g->host_small[0];
  return NLP_OK;
}

nlp_status nlp_last_common(nlp_graph* g, uint64_t* common) {
  if (!g || !common) return NLP_ERR_INVALID;
  if (!g->last_out && g->last_n) return NLP_ERR_INVALID;
  return nlp_count_common_device(g, (const nlp_edge*)g->last_out, g->last_n, common, g->last_stream);
}

nlp_status nlp_select_edges_device(nlp_graph* g, const nlp_edge* d_in, uint64_t n, uint64_t max_edges,
                                   nlp_edge* d_out, uint64_t* out_count, void* stream) {
  if (g && g->is_group) return nlp_select_edges_device(g->members[0], d_in, n, max_edges, d_out, out_count, stream);
  if (!g || !out_count || (n && !d_in) || (max_edges && !d_out)) return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  hipStream_t st = stream ? (hipStream_t)stream : g->stream;
  if (!stream && hipDeviceSynchronize() != hipSuccess) return NLP_ERR_DEVICE;
  Cands C;
  if (n) {
    uint32_t *ck, *cu, *cw;
    float* cs;
    TRY(wsget(g->ws, B_CKEY, n, &ck));
    TRY(wsget(g->ws, B_CU, n, &cu));
    TRY(wsget(g->ws, B_CW, n, &cw));
    TRY(wsget(g->ws, B_CS, n, &cs));
    LAUNCH(k_split_edges, n, st, (const EdgeOut*)d_in, n, ck, cu, cw, cs);
    TRY(hipGetLastError());
    C.n = n;
  }
  nlp_status s = prune_to(g, C, max_edges, st);
  if (s != NLP_OK) return s;
  s = order_v1(g, C, (EdgeOut*)d_out, st);
  if (s != NLP_OK) return s;
  TRY(hipStreamSynchronize(st));
  *out_count = C.n;
  return NLP_OK;
}

nlp_status nlp_merge_blocks_device(nlp_graph* g, const nlp_edge* d_blocks, uint64_t stride, uint32_t nblocks,
                                   uint64_t max_edges, nlp_edge* d_out, uint64_t* out_count, void* stream) {
  if (g && g->is_group)
    return nlp_merge_blocks_device(g->members[0], d_blocks, stride, nblocks, max_edges, d_out, out_count, stream);
  if (!g || !out_count || !d_blocks || stride < 1 || nblocks < 1 || nblocks > 65535 || (max_edges && !d_out) ||
      (uint64_t)nblocks * stride >= (1ull << 32))  // merge ranks are 32-bit
    return NLP_ERR_INVALID;
  if (hipSetDevice(g->device) != hipSuccess) return NLP_ERR_DEVICE;
  hipStream_t st = stream ? (hipStream_t)stream : g->stream;
  if (!stream && hipDeviceSynchronize() != hipSuccess) return NLP_ERR_DEVICE;
  unsigned long long* c;
  TRY(wsget(g->ws, B_EVAL, 8, &c));
  TRY(hipMemsetAsync(c + 4, 0, 32, st));
  hipLaunchKernelGGL(k_merge_blocks_check, dim3(1), dim3(64), 0, st, (const EdgeOut*)d_blocks, stride, nblocks, c);
  TRY(hipGetLastError());
  if (max_edges && stride > 1) {
    const uint64_t gx = (stride - 1 + NT - 1) / NT;
    if (gx > 0x7fffffffull) return NLP_ERR_INVALID;
    uint32_t* keys;
    TRY(wsget(g->ws, B_MKEY, stride * nblocks, &keys));
    hipLaunchKernelGGL(k_merge_keys, dim3((unsigned)gx, nblocks), dim3(NT), 0, st, (const EdgeOut*)d_blocks, stride,
                       (const unsigned long long*)c, keys);
    TRY(hipGetLastError());
    const uint64_t tiles = (stride - 1 + MT_T - 1) / MT_T;
    uint64_t* bnd;
    TRY(wsget(g->ws, B_MBND, 4 * (uint64_t)nblocks * nblocks * tiles, &bnd));
    hipLaunchKernelGGL(k_merge_bounds, dim3(grid_full(4 * (uint64_t)nblocks * nblocks * tiles)), dim3(NT), 0, st,
                       (const EdgeOut*)d_blocks, stride, nblocks, tiles, (const unsigned long long*)c,
                       (const uint32_t*)keys, bnd);
    TRY(hipGetLastError());
    hipLaunchKernelGGL(k_merge_blocks, dim3((unsigned)tiles, nblocks), dim3(MT_NT), 0, st, (const EdgeOut*)d_blocks,
                       stride, nblocks, max_edges, (const unsigned long long*)c, (const uint32_t*)keys,
                       (const uint64_t*)bnd, (EdgeOut*)d_out, debug_on() ? c + 4 : nullptr);
    TRY(hipGetLastError());
  }
  TRY(hipMemcpyAsync(g->host_small, c, 64, hipMemcpyDeviceToHost, st));
  TRY(hipStreamSynchronize(st));
  if (debug_on())
    fprintf(stderr, "nlp: merge windows %llu mean len %.1f beyond LDS %llu distinct keys/tile %.1f\n",
            (unsigned long long)g->host_small[4], g->host_small[4] ? (double)g->host_small[5] / g->host_small[4] : 0.0,
            (unsigned long long)g->host_small[6],
            g->host_small[4] ? (double)g->host_small[7] * (nblocks - 1) / g->host_small[4] : 0.0);
  const uint64_t tot = g->host_small[0], mx = g->host_small[1], bad = g->host_small[2];
  if (bad) {
    *out_count = mx;
    return NLP_ERR_CAPACITY;
  }
  *out_count = std::min(tot, max_edges);
  return NLP_OK;
}

const char* nlp_status_string(nlp_status s) {
  switch (s) {
    case NLP_OK: return "ok";
    case NLP_ERR_INVALID: return "invalid argument";
    case NLP_ERR_DEVICE: return "HIP device error";
    case NLP_ERR_NOMEM: return "out of memory";
    case NLP_ERR_NODEVICE: return "no gfx950 device";
    case NLP_ERR_CAPACITY: return "output buffer too small";
    case NLP_ERR_RETRY: return "an asynchronous prediction needs a synchronous redo";
  }
  return "unknown status";
}

const char* nlp_metric_name(nlp_metric m) {
  static const char* names[] = {"CommonNeighbors", "JaccardCoefficient", "SorensenIndex",
                                "SaltonCosineSimilarity", "HubPromoted", "HubDepressed",
                                "LeichtHolmeNermanScore", "AdamicAdarCoefficient",
                                "ResourceAllocationScore"};
  return ((int)m >= 0 && (int)m <= 8) ? names[(int)m] : "unknown";
}

int nlp_version(void) { return 100; }

}  // extern "C"
