// hashpath.hpp -- path 3: source-centric hash accumulation for large wedge counts.
//
// Reference: predictLinksWithIntersectionLoopOmpU (/root/reference/inc/predict.hxx:284-339).
// Per source u the reference walks every first-hop v (hub filter deg v <= H,
// predict.hxx:298-301), every second-hop w > u of N(v) (ft, 292-296), and
// accumulates into a dense per-thread table V[S] (predictScanEdges[Basic]U,
// 153-179); it then zeroes u and N(u) (306-307) and scores every touched w.
//
// Here one wave (small rows) or one 1024-thread workgroup (large rows) owns a
// source row and accumulates the wedges of that row in an open-addressing hash
// table: in LDS while the row's wedge count fits (W(u) <= 4096), in a
// per-workgroup global slab beyond.  Nothing proportional to the wedge count is
// ever materialised, so hub thresholds up to IHub (H = 0) run in bounded
// memory; the wedge scan is flattened over the row's surviving intermediates
// (a prefix of their degrees in LDS, a binary search per wedge) so that lanes
// stay busy whatever the degree mix.
//
// Exactness.  Counts are order-free.  Adamic-Adar / Resource-Allocation add
// (float)((double)acc + c_v) in the order of v in N(u) (predict.hxx:788, 828),
// which an unordered hash cannot reproduce, so the table keeps the count and
// the last inserting v: a count of 1 scores (float)(0.0 + c_v) directly, and a
// count >= 2 re-walks the intersection N(u) x I(w) (I = transposed adjacency,
// v in I(w) <=> w in N(v), with multiplicities) in ascending v -- the same
// sequence of additions as the reference.
//
// Candidates are emitted unordered (wave-aggregated atomics) into a buffer
// shared by the chunks of source rows; between chunks the host prunes the
// buffer to the canonical top k (key desc, u asc, w asc) and raises the
// emission threshold tau to the k-th key: later chunks hold larger u, so a
// later candidate with key <= tau can never enter the top k.
#pragma once
#include "group.hpp"

namespace nlp {

constexpr uint32_t HP_EMPTY = 0xffffffffu;
constexpr uint32_t HP_EXCL = 0x80000000u;   // count bit: w in N(u) (first-order exclusion)
constexpr uint32_t HP_CMASK = 0x7fffffffu;
constexpr int HP_WT = 1024;                 // wave table entries (bin 0)
constexpr uint64_t HP_B0_MAX = HP_WT / 2;   // bin 0: W(u) <= 512
constexpr uint64_t HP_B0_DEG = 1024;        //        and deg(u) <= 1024
constexpr int HP_BNT = 1024;                // workgroup size of the block bins
constexpr int HP_BT = 8192;                 // LDS table entries (bin 1)
constexpr uint64_t HP_B1_MAX = HP_BT / 2;   // bin 1: W(u) <= 4096
constexpr uint64_t HP_B2_MAX = 1ull << 19;  // bin 2: W(u) <= 2^19, bin 3: the rest (both k_hp_part)
constexpr int HP_NBINS = 4;

// per-chunk counters (u64)
// HPC_HOTB: algorithmic bytes of the chunk's k_hp_batch launch, counted by the kernel;
// HPC_PAD: padding entries written into the unused tails of emission windows (hp_flush)
// HPC_BIGW: wedges of the hub pass's HH_BIG items (AA / RA hash tables with the ordered re-walk; diagnostic)
enum { HPC_EMIT = 0, HPC_CAND = 1, HPC_NAN = 2, HPC_WEDGE = 3, HPC_ERR = 4, HPC_HOTB = 5, HPC_PAD = 6, HPC_BIGW = 7,
       HPC_NCTR = 8 };

struct HpArgs {
  GraphView g;
  uint64_t S;
  uint32_t H;
  uint32_t ctn;       // entries of g.ctab (max degree + 1): the AA / RA contribution table
  int metric;
  float min_score;
  uint32_t* ckey;     // candidate columns (score key, u, w, score)
  uint32_t* cu;
  uint32_t* cw;
  float* cs;
  uint64_t base;      // first free slot
  uint64_t cap;       // free slots from base on
  const int64_t* tau; // emit only key > *tau
  unsigned long long* ctr;
  // small H: the surviving first hops of every source of the range (S(u) =
  // {v in N(u) : deg v <= H}, multiplicities kept, any order), so a row walks
  // S(u) instead of all of N(u) with a degree gather per entry (null: N(u))
  const uint64_t* soff;  // [nU + 1], indexed by u - sua: S(u) = skeys[soff[u - sua], + |S(u)|)
  const uint32_t* scn;   // |S(u)|, indexed by u - sua (null: soff[u - sua + 1] - soff[u - sua])
  const uint32_t* skeys;
  uint64_t sua;
  int ssorted;  // S(u) in N(u)'s (ascending) order: the AA / RA row kernels skip their sort
  const uint32_t* kdeg;  // deg keys[e] per adjacency entry (null: none; KD row kernels)
  const uint64_t* sdo;   // S(u) entries packed deg v << 48 | n << HP_SDO_SH | o, [o, o + n) = N(v) above u (null: none)
  const uint32_t* xs;    // per row: entries of N(u) at or below u (null: none; the exclusion starts after them)
  unsigned long long* ph;  // diagnostic (NLP_TRACE_BATCH=1 / NLP_TRACE_HUB=1): phase ticks, 100 MHz (null: off)
  uint32_t win;            // k_hp_batch's emission window in slots (0: a reservation per flush; padding in HPC_PAD)
  uint32_t uxf;            // rows whose exclusion slice exceeds uxf x W test the membership table (HP_UX_OFF: never)
};

// xs[u] = the number of entries of N(u) that are <= u (one binary search per row)
__global__ void k_hp_xs(const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys, uint64_t S,
                        uint32_t* __restrict__ xs) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < S; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t lo = off[u], hi = off[u + 1];
    const uint64_t o = lo;
    while (lo < hi) {
      const uint64_t m = (lo + hi) >> 1;
      if (keys[m] <= (uint32_t)u) lo = m + 1; else hi = m;
    }
    xs[u] = (uint32_t)(lo - o);
  }
}
constexpr int HP_SDO_SH = 40;  // offsets < 2^40 (guarded at the list build)

// S(u)'s start in skeys / sdo and its length (the class-ordered short lists
// leave gaps between rows: lengths from scn)
__device__ __forceinline__ uint64_t hp_slen(const HpArgs& a, uint32_t u, uint64_t s0) {
  return a.scn ? (uint64_t)a.scn[u - a.sua] : a.soff[u - a.sua + 1] - s0;
}

// A row's first-hop list: S(u) when the survivor lists exist, else N(u).
__device__ __forceinline__ void hp_first_hops(const HpArgs& a, uint32_t u, uint64_t o0, uint64_t du,
                                              const uint32_t** list, uint64_t* n) {
  if (a.soff) {
    const uint64_t s0 = a.soff[u - a.sua];
    *list = a.skeys + s0;
    *n = hp_slen(a, u, s0);
  } else {
    *list = a.g.keys + o0;
    *n = du;
  }
}

__device__ __forceinline__ bool hp_surv(uint32_t d, uint32_t H) { return d > 0 && (H == 0 || d <= H); }

__device__ __forceinline__ uint32_t hp_hash(uint32_t w, int shift) { return (w * 0x9E3779B1u) >> shift; }

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

__device__ __forceinline__ int log2_ceil(uint64_t x) {
  int b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}

// ---------------------------------------------------------------- table access
// LDS tables use plain loads; global slabs go through agent-scope atomics so
// that no stale L1 line of a previous row is ever read.
template <bool GLOBAL>
__device__ __forceinline__ uint32_t tload(const uint32_t* p) {
  if (GLOBAL) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *(volatile const uint32_t*)p;
}
template <bool GLOBAL>
__device__ __forceinline__ void tstore(uint32_t* p, uint32_t v) {
  if (GLOBAL) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *(volatile uint32_t*)p = v;
}

// A table: keys (HP_EMPTY = free), counts (HP_EXCL bit = w in N(u)) and, for
// AA / RA, the smallest and largest contributing v (empty: ~0 / 0).
struct HpTable {
  uint32_t* k;
  uint32_t* c;
  uint32_t* vmin;
  uint32_t* vmax;
};

// Tables are sized for at most half load, so a probe sequence always ends; a
// full table (a sizing bug) raises HPC_ERR instead of spinning.
template <bool GLOBAL, bool CUSTOM>
__device__ __forceinline__ void hp_insert(const HpTable& t, uint32_t mask, int shift, uint32_t w, uint32_t v,
                                          unsigned long long* err) {
  uint32_t h = hp_hash(w, shift);
  for (uint32_t probe = 0;; ++probe) {
    if (probe > mask) { atomicOr(err, 1ull); return; }
    uint32_t cur = tload<GLOBAL>(&t.k[h]);
    if (cur == HP_EMPTY) {
      cur = atomicCAS(&t.k[h], HP_EMPTY, w);
      if (cur == HP_EMPTY) cur = w;
    }
    if (cur == w) {
      atomicAdd(&t.c[h], 1u);
      if (CUSTOM) {
        atomicMin(&t.vmin[h], v);
        atomicMax(&t.vmax[h], v);
      }
      return;
    }
    h = (h + 1) & mask;
  }
}

template <bool GLOBAL>
__device__ __forceinline__ void hp_mark(const HpTable& t, uint32_t mask, int shift, uint32_t x) {
  uint32_t h = hp_hash(x, shift);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const uint32_t cur = tload<GLOBAL>(&t.k[h]);
    if (cur == x) { atomicOr(&t.c[h], HP_EXCL); return; }
    if (cur == HP_EMPTY) return;
    h = (h + 1) & mask;
  }
}

// Read entry i and reset it to empty.
template <bool GLOBAL, bool CUSTOM>
__device__ __forceinline__ uint32_t hp_take(const HpTable& t, uint32_t i, uint32_t* c, uint32_t* v0, uint32_t* v1) {
  const uint32_t w = tload<GLOBAL>(&t.k[i]);
  if (w != HP_EMPTY) {
    *c = tload<GLOBAL>(&t.c[i]);
    tstore<GLOBAL>(&t.k[i], HP_EMPTY);
    tstore<GLOBAL>(&t.c[i], 0u);
    if (CUSTOM) {
      *v0 = tload<GLOBAL>(&t.vmin[i]);
      *v1 = tload<GLOBAL>(&t.vmax[i]);
      tstore<GLOBAL>(&t.vmin[i], HP_EMPTY);
      tstore<GLOBAL>(&t.vmax[i], 0u);
    }
  }
  return w;
}

// Exact Adamic-Adar / Resource-Allocation value of (u, w) with n >= 3
// contributions: the additions of predict.hxx:788/828 in ascending v over
// N(u) x I(w) (multiplicities multiply), iterating the shorter list.
__device__ float hp_ordered_sum(const HpArgs& a, uint32_t u, uint32_t w, uint32_t n) {
  const uint64_t ou = a.g.off[u], tw = a.g.toff[w];
  const uint32_t na = (uint32_t)(a.g.off[u + 1] - ou), nb = (uint32_t)(a.g.toff[w + 1] - tw);
  const bool iter_a = na <= nb;
  const uint32_t* X = iter_a ? a.g.keys + ou : a.g.tkeys + tw;
  const uint32_t* Y = iter_a ? a.g.tkeys + tw : a.g.keys + ou;
  const uint32_t nx = iter_a ? na : nb, ny = iter_a ? nb : na;
  float acc = 0.0f;
  uint32_t done = 0, lo = 0;
  for (uint32_t i = 0; i < nx && done < n; ++i) {
    const uint32_t v = X[i];
    const uint32_t d = a.g.deg[v];
    if (!hp_surv(d, a.H)) continue;
    uint32_t l = lo, h = ny;
    while (l < h) {
      const uint32_t m = (l + h) >> 1;
      if (Y[m] < v) l = m + 1; else h = m;
    }
    lo = l;
    uint32_t m = 0;
    while (l + m < ny && Y[l + m] == v) ++m;
    const double c = a.g.ctab[d];
    for (uint32_t q = 0; q < m; ++q) acc = (float)((double)acc + c);
    done += m;
  }
  return acc;
}

// Score of a table entry.  AA / RA: one contribution is c(vmin); two are
// c(vmin) then c(vmax) (ascending v, equal when one v contributes twice);
// three or more re-walk the intersection.
template <bool CUSTOM>
__device__ __forceinline__ float hp_score(const HpArgs& a, uint32_t u, uint64_t du, uint32_t w, uint32_t c,
                                          uint32_t v0, uint32_t v1) {
  const bool ex = (c & HP_EXCL) != 0;
  const uint32_t n = c & HP_CMASK;
  if (!CUSTOM) return score_basic(a.metric, ex ? 0u : n, du, (uint64_t)a.g.deg[w]);
  if (ex) return 0.0f;
  if (n <= 2) {
    float acc = (float)((double)0.0f + a.g.ctab[a.g.deg[v0]]);
    if (n == 2) acc = (float)((double)acc + a.g.ctab[a.g.deg[v1]]);
    return acc;
  }
  return hp_ordered_sum(a, u, w, n);
}

// Count tables that also hold the second hop's degree (KD row kernels): count
// in bits [0, CB), min(deg w, 2^(31 - CB) - 1) above it (added once, by the
// thread whose CAS creates the entry), HP_EXCL on top.  A saturated degree is
// gathered at the drain.
template <int CB>
__device__ __forceinline__ void hp_insert_kd(const HpTable& t, uint32_t mask, int shift, uint32_t key, uint32_t dw,
                                             unsigned long long* err) {
  constexpr uint32_t DSAT = (1u << (31 - CB)) - 1u;
  uint32_t h = hp_hash(key, shift);
  for (uint32_t probe = 0;; ++probe) {
    if (probe > mask) { atomicOr(err, 1ull); return; }
    uint32_t cur = *(volatile uint32_t*)&t.k[h];
    bool mine = false;
    if (cur == HP_EMPTY) {
      cur = atomicCAS(&t.k[h], HP_EMPTY, key);
      if (cur == HP_EMPTY) { cur = key; mine = true; }
    }
    if (cur == key) {
      atomicAdd(&t.c[h], 1u + (mine ? (dw < DSAT ? dw : DSAT) << CB : 0u));
      return;
    }
    h = (h + 1) & mask;
  }
}

template <int CB>
__device__ __forceinline__ uint32_t hp_kd_deg(const GraphView& g, uint32_t c, uint32_t w) {
  constexpr uint32_t DSAT = (1u << (31 - CB)) - 1u;
  const uint32_t d = (c & HP_CMASK) >> CB;
  return d < DSAT ? d : g.deg[w];
}

// ---------------------------------------------------------------- ordered AA / RA accumulation
// The row kernels of bins 0 and 1 (k_hp_batch, k_hp_wave, k_hp_block) add the
// Adamic-Adar / Resource-Allocation contributions in the reference's order
// instead of re-walking intersections.  With a row's first hops in ascending v
// (N(u) is sorted; the survivor lists S(u) are sorted in LDS first), the
// flattened wedge index j runs in the order of predict.hxx:153-179 (v ascending
// over N(u), then N(v)) for every w.  Wedges are taken in steps of one per
// thread, j ascending with the thread index, steps one after another; within
// a step, threads that hit the same entry add in thread order: each pending
// thread posts a token (round << TB | reversed thread index) to the entry's
// owner word with atomicMax, the winner -- the lowest pending thread of that
// entry -- adds (float)((double)acc + c_v), the others retry in the next round
// (one round unless a step holds the same w twice).  The table's count word
// holds the float accumulator (the sign bit, HP_EXCL, is the exclusion mark: an
// accumulator is never negative) and vmin the owner tokens (0 when free).
__device__ __forceinline__ uint32_t ho_find(const HpTable& t, uint32_t mask, int shift, uint32_t key,
                                            unsigned long long* err) {
  uint32_t h = hp_hash(key, shift);
  for (uint32_t probe = 0;; ++probe) {
    if (probe > mask) { atomicOr(err, 1ull); return 0u; }
    uint32_t cur = *(volatile uint32_t*)&t.k[h];
    if (cur == HP_EMPTY) {
      cur = atomicCAS(&t.k[h], HP_EMPTY, key);
      if (cur == HP_EMPTY) cur = key;
    }
    if (cur == key) return h;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ void ho_apply(const HpTable& t, uint32_t h, double c) {
  const float a = __uint_as_float(*(volatile uint32_t*)&t.c[h]);
  *(volatile uint32_t*)&t.c[h] = __float_as_uint((float)((double)a + c));
}

// one wave's step (every lane calls it; pend = this lane has a wedge)
__device__ __forceinline__ void ho_add_wave(const HpTable& t, bool pend, uint32_t h, double c, uint32_t* round) {
  const uint32_t lane = (uint32_t)lane_id();
  while (__ballot(pend)) {
    const uint32_t tok = (*round << 6) | (63u - lane);
    if (pend) atomicMax(&t.vmin[h], tok);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    if (pend && *(volatile uint32_t*)&t.vmin[h] == tok) {
      ho_apply(t, h, c);
      pend = false;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    ++*round;
  }
}

// one workgroup's step (HP_BNT = 1024 threads, every thread calls it)
template <int TB = 10>  // a workgroup of 2^TB threads
__device__ __forceinline__ void ho_add_block(const HpTable& t, bool pend, uint32_t h, double c, uint32_t* round) {
  const uint32_t tid = threadIdx.x;
  while (__syncthreads_or(pend)) {
    const uint32_t tok = (*round << TB) | ((1u << TB) - 1u - tid);
    if (pend) atomicMax(&t.vmin[h], tok);
    __syncthreads();
    if (pend && *(volatile uint32_t*)&t.vmin[h] == tok) {
      ho_apply(t, h, c);
      pend = false;
    }
    ++*round;
  }
}

// Read entry i and reset it (key, accumulator, owner).
__device__ __forceinline__ uint32_t ho_take(const HpTable& t, uint32_t i, uint32_t* c) {
  const uint32_t w = *(volatile uint32_t*)&t.k[i];
  if (w != HP_EMPTY) {
    *c = *(volatile uint32_t*)&t.c[i];
    *(volatile uint32_t*)&t.k[i] = HP_EMPTY;
    *(volatile uint32_t*)&t.c[i] = 0u;
    *(volatile uint32_t*)&t.vmin[i] = 0u;
  }
  return w;
}

// score of an ordered entry: 0 when w is in N(u) (predict.hxx:306-307), else the sum
__device__ __forceinline__ float ho_score(uint32_t c) { return (c & HP_EXCL) ? 0.0f : __uint_as_float(c); }

// Ascending bitonic sort of n (a power of two, >= 2) words in LDS by one wave.
__device__ __forceinline__ void wave_bitonic_u32(uint32_t* s, uint32_t n) {
  const uint32_t lane = (uint32_t)lane_id();
  for (uint32_t k = 2; k <= n; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = lane; i < n / 2; i += 64) {
        const uint32_t lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
        const uint32_t x = s[lo], y = s[hi];
        if ((x > y) == ((lo & k) == 0)) {
          s[lo] = y;
          s[hi] = x;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
}

// The same over a workgroup of HP_BNT threads.
__device__ __forceinline__ void block_bitonic_u32(uint32_t* s, uint32_t n) {
  for (uint32_t k = 2; k <= n; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < n / 2; i += blockDim.x) {
        const uint32_t lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
        const uint32_t x = s[lo], y = s[hi];
        if ((x > y) == ((lo & k) == 0)) {
          s[lo] = y;
          s[hi] = x;
        }
      }
      __syncthreads();
    }
}

__device__ __forceinline__ uint32_t pow2_at_least(uint32_t n) {
  uint32_t p = 2;
  while (p < n) p <<= 1;
  return p;
}

// ---------------------------------------------------------------- emission
// Per-wave staging of emitted candidates in LDS: one global atomic per
// HP_STG candidates instead of one per wave and iteration (a single counter
// hammered by every wave of the chip serialises at one L2 channel).  The
// candidate / NaN counts stay in registers until the kernel ends.
constexpr int HP_STG = 128;

// A row whose exclusion slice (the entries of N(u) above u) exceeds HB_XF
// times its wedge bound tests its table entries in the per-graph membership
// table instead (one 64-byte line per entry, kernels.hpp et_has) of marking
// the slice: a high-degree row with a few low-degree neighbours would read
// thousands of keys for a handful of entries.  C4 JAC H=16, row batches: 18.8
// ms with marks only, 18.8 / 16.4 / 14.8 / 14.6 / 14.2 ms at factors 8 / 4 / 2 /
// 1 / 0 (every row by the table); uk-2005's neighbourhoods favour the marks (C3
// AA H=16: 106 / 100 / 97 ms at 1 / 2 / 4): 2 is within 1 % of the best on
// both.
constexpr uint64_t HB_XF = 2;
constexpr uint32_t HP_UX_OFF = 0xffffffffu;
__device__ __forceinline__ bool hp_use_etab(const HpArgs& a, uint64_t dx, uint64_t W) {
  return a.g.etab && a.uxf != HP_UX_OFF && dx > (uint64_t)a.uxf * W;
}

struct HpStage {
  uint32_t* u;
  uint32_t* w;
  float* s;
  uint32_t cap;   // entries per array
  uint32_t n;     // wave-uniform fill
  uint64_t cand, nan;
  uint64_t out;   // candidates written (wave-uniform; the batch kernel's algorithmic bytes)
  // emission window (wave-uniform; wend > 0: windowed): slots [wpos, wend)
  // reserved with one atomic per HP_WIN candidates, the unused tail padded
  uint64_t wpos, wend;
  bool win;
  uint64_t pad;
};
// Emission windows.  Every wave of every path-4 kernel reserving each flush
// on ONE counter serialises at the memory side (C4 JAC H=16: 2.2 M
// reservations, ~7 ms of the row batches); the row batches' persistent waves
// reserve a.win slots at a time (sized by the host to a fraction of a wave's
// expected emissions, at most HP_WIN) and pad what a window does not use with
// entries that can never be selected (score key 0, u = w = 0xffffffff: last of
// every tie), counted in HPC_PAD and dropped by the prune.
constexpr uint64_t HP_WIN = 4096;
constexpr uint32_t HP_PADID = 0xffffffffu;

// Orders one wave's LDS accesses across lanes (staging, scan arrays, LDS
// tables).  A wavefront-scope fence emits no instruction and the wave barrier
// carries no memory semantics, so the machine scheduler may still move plain
// DS reads and writes across them; a workgroup-scope fence is a real
// s_waitcnt that nothing is scheduled across.
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
}

// padding entries in slots [p0, p1) of the chunk's emission region
__device__ __forceinline__ void hp_pad(const HpArgs& a, uint64_t p0, uint64_t p1) {
  for (uint64_t p = p0 + lane_id(); p < p1; p += 64)
    if (p < a.cap) {
      const uint64_t q = a.base + p;
      a.ckey[q] = 0u;
      a.cu[q] = HP_PADID;
      a.cw[q] = HP_PADID;
      a.cs[q] = __uint_as_float(0x7fc00000u);
    }
}

__device__ __forceinline__ void hp_flush(HpStage& st, const HpArgs& a) {
  if (st.n == 0) return;
  wave_sync_lds();
  const int lane = lane_id();
  unsigned long long pos = 0;
  if (st.win) {
    if (st.wpos + st.n > st.wend) {  // a new window; the old one's tail padded
      hp_pad(a, st.wpos, st.wend);
      st.pad += st.wend - st.wpos;
      const uint64_t wsz = (uint64_t)a.win > st.n ? (uint64_t)a.win : st.n;
      if (lane == 0) pos = atomicAdd(&a.ctr[HPC_EMIT], (unsigned long long)wsz);
      st.wpos = __shfl(pos, 0, 64);
      st.wend = st.wpos + wsz;
    }
    pos = st.wpos;
    st.wpos += st.n;
  } else {
    if (lane == 0) pos = atomicAdd(&a.ctr[HPC_EMIT], (unsigned long long)st.n);
    pos = __shfl(pos, 0, 64);
  }
  for (uint32_t i = lane; i < st.n; i += 64) {
    const uint64_t p = pos + i;
    if (p < a.cap) {
      const uint64_t q = a.base + p;
      a.ckey[q] = score_key(st.s[i]);  // recomputed: 12 B per staged entry
      a.cu[q] = st.u[i];
      a.cw[q] = st.w[i];
      a.cs[q] = st.s[i];
    }
  }
  wave_sync_lds();
  st.out += st.n;
  st.n = 0;
}

// Candidate filter (predict.hxx:309-311: score <= minScore skips, NaN passes)
// and emission above tau; every active lane of the wave calls it.
__device__ __forceinline__ void hp_emit(HpStage& st, const HpArgs& a, bool valid, float s, uint32_t u, uint32_t w,
                                        int64_t tau) {
  const bool cand = valid && !(s <= a.min_score) && !f2_drop(a.g, u, w);
  st.cand += cand ? 1 : 0;
  st.nan += (cand && s != s) ? 1 : 0;
  const uint32_t key = cand ? score_key(s) : 0u;
  const bool out = cand && (int64_t)key > tau;
  const uint64_t mo = __ballot(out);
  if (!mo) return;
  const uint32_t n = (uint32_t)__popcll(mo);
  if (st.n + n > st.cap) hp_flush(st, a);
  if (out) {
    const uint32_t i = st.n + (uint32_t)__popcll(mo & ((1ull << lane_id()) - 1));
    st.u[i] = u;
    st.w[i] = w;
    st.s[i] = s;
  }
  st.n += n;
}

__device__ __forceinline__ void hp_finish(HpStage& st, const HpArgs& a, uint64_t wedges) {
  hp_flush(st, a);
  if (st.win) {  // the last window's tail
    hp_pad(a, st.wpos, st.wend);
    st.pad += st.wend - st.wpos;
    st.wpos = st.wend;
  }
  const uint64_t c = wave_sum(st.cand), n = wave_sum(st.nan), wd = wave_sum(wedges);
  if (lane_id() == 0) {
    if (c) atomicAdd(&a.ctr[HPC_CAND], (unsigned long long)c);
    if (n) atomicAdd(&a.ctr[HPC_NAN], (unsigned long long)n);
    if (wd) atomicAdd(&a.ctr[HPC_WEDGE], (unsigned long long)wd);
    if (st.pad) atomicAdd(&a.ctr[HPC_PAD], (unsigned long long)st.pad);
  }
}

// ---------------------------------------------------------------- latency batching
// Every loop below does a dependent global load per item (a key of N(v), a
// degree, a scratch word) and then LDS work on it.  Issued one item at a time
// a lane waits a full memory round trip per item; here each lane first issues
// the loads of HP_UN items (their addresses from LDS searches, which do not
// wait on the outstanding global loads: separate counters), then consumes them.
constexpr int HP_UN = 2;

// The wedges of one block of first-hop entries: wedge j belongs to the entry
// whose inclusive length prefix s_incl first exceeds j (NS entries, searched in
// LDS); f(w, v) for every wedge, HP_UN per lane in flight.  stride = the
// threads sharing the block (64: a wave; HP_BNT: a workgroup), t = this
// thread's index among them.
// ALL: f(ok, w, entry) on every thread (convergent; entry = the first-hop index).
// KD: f(w, v, deg w) with the degree loaded beside the key from kd[].
template <int NS, bool ALL = false, bool KD = false, typename IT, typename F>
__device__ __forceinline__ void hp_wedges(uint64_t total, uint32_t t, uint32_t stride, const IT* s_incl,
                                          const uint64_t* s_start, const uint32_t* s_iv, const uint32_t* keys, F f,
                                          const uint32_t* kd = nullptr) {
  for (uint64_t j0 = 0; j0 < total; j0 += (uint64_t)stride * HP_UN) {
    uint32_t w[HP_UN], v[HP_UN], dw[HP_UN];
    bool ok[HP_UN];
#pragma unroll
    for (int q = 0; q < HP_UN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * stride + t;
      ok[q] = j < total;
      uint32_t lo = 0, hi = NS - 1;  // first entry o with s_incl[o] > j
      while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if ((uint64_t)s_incl[m] > j) hi = m; else lo = m + 1;
      }
      const uint64_t ex = lo ? (uint64_t)s_incl[lo - 1] : 0ull;
      v[q] = ALL ? lo : s_iv[lo];
      const uint64_t at = ok[q] ? s_start[lo] + (j - ex) : 0ull;
      w[q] = keys[at];
      if constexpr (KD) dw[q] = kd[at];
    }
#pragma unroll
    for (int q = 0; q < HP_UN; ++q) {
      if constexpr (ALL) f(ok[q], w[q], v[q]);
      else if constexpr (KD) { if (ok[q]) f(w[q], v[q], dw[q]); }
      else if (ok[q]) f(w[q], v[q]);
    }
  }
}

// n consecutive words src[0..n): f(x) for each, HP_UN per lane in flight
template <typename F>
__device__ __forceinline__ void hp_stream(const uint32_t* src, uint64_t n, uint32_t t, uint32_t stride, F f) {
  for (uint64_t i0 = 0; i0 < n; i0 += (uint64_t)stride * HP_UN) {
    uint32_t x[HP_UN];
#pragma unroll
    for (int q = 0; q < HP_UN; ++q) {
      const uint64_t i = i0 + (uint64_t)q * stride + t;
      x[q] = src[i < n ? i : 0ull];
    }
#pragma unroll
    for (int q = 0; q < HP_UN; ++q)
      if (i0 + (uint64_t)q * stride + t < n) f(x[q]);
  }
}

// Take, score and emit every entry of a table of T slots (T a multiple of
// 64): the slots of HP_UN rounds first (LDS or slab), then their degree loads
// (count metrics) in flight together, then the scores; every thread of the
// caller runs every round (hp_emit ballots per wave).
// ORD: an ordered AA / RA table (LDS only, see ho_add_wave).  KCB > 0: a KD
// count table (hp_insert_kd<KCB>: deg w in the count word).
template <bool GLOBAL, bool CUSTOM, int UN = HP_UN, bool ORD = false, int KCB = 0>
__device__ __forceinline__ void hp_drain(const HpTable& tb, uint32_t T, uint32_t t, uint32_t stride, HpStage& sg,
                                         const HpArgs& a, uint32_t u, uint64_t du, int64_t tau, bool ux = false) {
  T = __builtin_amdgcn_readfirstlane(T);
  for (uint32_t i0 = 0; i0 < T; i0 += stride * UN) {
    uint32_t w[UN], c[UN], v0[UN], v1[UN], dw[UN];
    const uint32_t nq = min((uint32_t)UN, (T - i0 + stride - 1) / stride);  // steps inside the table (uniform)
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      if ((uint32_t)q >= nq) break;
      const uint32_t i = i0 + (uint32_t)q * stride + t;
      c[q] = v0[q] = v1[q] = 0;
      if (ORD) w[q] = i < T ? ho_take(tb, i, &c[q]) : HP_EMPTY;
      else w[q] = i < T ? hp_take<GLOBAL, CUSTOM>(tb, i, &c[q], &v0[q], &v1[q]) : HP_EMPTY;
    }
    if (ux) {  // the first-order exclusion by the membership table (no marks were made), two probes in flight
#pragma unroll
      for (int q0 = 0; q0 < UN; q0 += 2) {
        uint64_t ek[2];
        bool ea[2], er[2];
#pragma unroll
        for (int z = 0; z < 2; ++z) {
          const int q = q0 + z;
          ea[z] = q < UN && (uint32_t)q < nq && w[q] != HP_EMPTY;
          ek[z] = ea[z] ? ((uint64_t)u << 32 | w[q]) : 0ull;
        }
        et_has_n<2>(a.g.etab, a.g.etbits, ek, ea, er);
#pragma unroll
        for (int z = 0; z < 2; ++z)
          if (q0 + z < UN && er[z]) c[q0 + z] |= HP_EXCL;
      }
    }
    if (ORD) {
#pragma unroll
      for (int q = 0; q < UN; ++q) {
        if ((uint32_t)q >= nq) break;
        hp_emit(sg, a, w[q] != HP_EMPTY, ho_score(c[q]), u, w[q], tau);
      }
      continue;
    }
    if (!CUSTOM) {
      // deg w for the score (Common Neighbours needs none: no gather per entry)
      const bool need_dw = a.metric != M_CN;
#pragma unroll
      for (int q = 0; q < UN; ++q) {
        if ((uint32_t)q >= nq) break;
        const uint32_t wq = w[q] != HP_EMPTY ? w[q] : 0u;
        if constexpr (KCB > 0) dw[q] = hp_kd_deg<KCB>(a.g, c[q], wq);
        else dw[q] = need_dw ? a.g.deg[wq] : 0u;
      }
    }
    constexpr uint32_t CM = KCB > 0 ? (1u << KCB) - 1u : HP_CMASK;
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      if ((uint32_t)q >= nq) break;
      const bool valid = w[q] != HP_EMPTY;
      float s = 0.0f;
      if (valid) {
        if (CUSTOM) s = hp_score<true>(a, u, du, w[q], c[q], v0[q], v1[q]);
        else s = score_basic(a.metric, (c[q] & HP_EXCL) ? 0u : (c[q] & CM), du, (uint64_t)dw[q]);
      }
      hp_emit(sg, a, valid, s, u, w[q], tau);
    }
  }
}

__global__ void k_sum_deg2_above(const uint32_t* __restrict__ deg, uint64_t S, uint32_t above,
                                 unsigned long long* __restrict__ out) {
  unsigned long long s = 0;
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < S; v += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t d = deg[v];
    if (d > above) s += d * d;
  }
  s = wave_sum(s);
  if (lane_id() == 0 && s) atomicAdd(out, s);
}

// ---------------------------------------------------------------- binning
// W(u) = sum of deg v over surviving v in N(u): an upper bound of the row's
// wedges (w > u is not applied).  Edge-parallel, so hub rows cost no more than
// their entries: a wave takes HP_WR x 64 consecutive adjacency entries
// (coalesced keys, HP_WR independent degree gathers per lane in flight),
// locates each entry's row among the next 64 row ends (held one per lane,
// searched with lane permutes), sums per row in LDS and adds each row's
// partial sum with one global atomic.  wu must be zeroed first.
constexpr int HP_WR = 8;
constexpr uint64_t HP_WTILE = 64 * HP_WR;  // adjacency entries per wave tile

// Per graph: the row of the first entry of every wave tile (tile_row[t] = the
// row u with off[u] <= t * HP_WTILE < off[u + 1]), so that a tile finds its
// rows without a search.
__global__ void k_hp_tile_rows(const uint64_t* __restrict__ off, uint64_t S, uint32_t* __restrict__ tile_row) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < S; u += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = off[u], b = off[u + 1];
    for (uint64_t t = (a + HP_WTILE - 1) / HP_WTILE; t * HP_WTILE < b; ++t) tile_row[t] = (uint32_t)u;
  }
}

__global__ __launch_bounds__(NT) void k_hp_work_edges(GraphView g, uint32_t H, uint64_t ua, uint64_t nU, uint64_t e0,
                                                      uint64_t e1, const uint32_t* __restrict__ tile_row,
                                                      unsigned long long* __restrict__ wu) {
  __shared__ unsigned long long s_acc[NWAVE][64];
  const int lane = lane_id(), wv = wave_id();
  const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE;
  s_acc[wv][lane] = 0;
  for (uint64_t tile = t0 + (uint64_t)blockIdx.x * NWAVE + wv; tile < t1; tile += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t base = tile * HP_WTILE;
    const uint64_t tr = tile_row[tile];
    const uint64_t r0 = tr > ua ? tr - ua : 0;  // first row of the tile inside the range
    const uint64_t rl = r0 + lane;
    const uint64_t rend = rl < nU ? g.off[ua + rl + 1] : ~0ull;  // end of row r0 + lane
    const uint64_t last_end = __shfl(rend, 63, 64);
    uint32_t c[HP_WR];
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      c[i] = 0;
      if (e >= e0 && e < e1) {
        const uint32_t d = g.deg[g.keys[e]];
        c[i] = hp_surv(d, H) ? d : 0u;
      }
    }
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      // local row: the number of the 64 row ends <= e (every lane searches: lane permutes)
      int lo = 0, hi = 64;
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        const uint64_t v = __shfl(rend, m, 64);
        if (v <= e) lo = m + 1; else hi = m;
      }
      if (c[i] == 0) continue;
      if (e < last_end) {
        atomicAdd(&s_acc[wv][lo], (unsigned long long)c[i]);
      } else {  // more than 64 rows in this tile: search the offsets
        uint64_t a = r0, b = nU;
        while (b - a > 1) {
          const uint64_t m = (a + b) >> 1;
          if (g.off[ua + m] <= e) a = m; else b = m;
        }
        atomicAdd(&wu[a], (unsigned long long)c[i]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    const unsigned long long v = s_acc[wv][lane];
    if (v) {
      atomicAdd(&wu[rl], v);
      s_acc[wv][lane] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  }
}

// ---------------------------------------------------------------- survivor lists by degree classes
// Per graph: dcls[e] = min(deg keys[e], 255).  For H <= HP_DCLS_MAX the
// survivor lists S(u) = {v in N(u): 1 <= deg v <= H} of a range are the stream
// compaction of its entries by dcls -- coalesced bytes, no atomics, and S(u)
// keeps N(u)'s ascending order (the AA / RA row kernels then need no sort).
//   k_hp_dcls_rows8: per row (cnt << 40 | W) packed into wu, per tile its count
//   k_hp_unpack:    wu -> W(u), cnt -> |S(u)| (scanned into soff by the caller)
//   k_hp_dcls_fill: per tile, the surviving keys at the scanned tile offsets
// (deg u < 2^24 is required at graph build, so the packed count cannot carry
// into W's 40 bits: W <= 254 deg u).
constexpr uint32_t HP_DCLS_MAX = 254;

__device__ __forceinline__ bool hp_dsurv(uint32_t c, uint32_t H) { return c >= 1 && c <= H; }

// The same per-row (count, W) and tile counts with eight consecutive entries
// per lane (one 8-byte load of classes): a lane finds the row of its first
// entry once (six LDS steps) and walks forward over the row ends, adding runs
// of one row with one LDS atomic, instead of a search per entry.
__global__ __launch_bounds__(NT) void k_hp_dcls_rows8(GraphView g, const uint8_t* __restrict__ dcls, uint32_t H,
                                                      uint64_t ua, uint64_t nU, uint64_t e0, uint64_t e1,
                                                      const uint32_t* __restrict__ tile_row,
                                                      unsigned long long* __restrict__ wu, uint32_t* __restrict__ tcnt) {
  __shared__ unsigned long long s_acc[NWAVE][64];
  __shared__ uint64_t s_end[NWAVE][64];
  const int lane = lane_id(), wv = wave_id();
  const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE;
  s_acc[wv][lane] = 0;
  for (uint64_t tile = t0 + (uint64_t)blockIdx.x * NWAVE + wv; tile < t1; tile += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t base = tile * HP_WTILE;
    const uint64_t tr = tile_row[tile];
    const uint64_t r0 = tr > ua ? tr - ua : 0;
    const uint64_t rl = r0 + lane;
    s_end[wv][lane] = rl < nU ? g.off[ua + rl + 1] : ~0ull;
    wave_sync_lds();
    const uint64_t last_end = s_end[wv][63];
    const uint64_t eb = base + (uint64_t)lane * 8;  // this lane's 8 entries
    uint64_t word = 0;
    if (eb + 8 <= e1 && eb >= e0) word = *(const uint64_t*)(dcls + eb);
    else
      for (int q = 0; q < 8; ++q)
        if (eb + q >= e0 && eb + q < e1) word |= (uint64_t)dcls[eb + q] << (8 * q);
    uint32_t tc = 0;
    int idx = 0;  // local row of the current entry: the number of row ends <= e
#pragma unroll
    for (uint32_t bit = 32; bit > 0; bit >>= 1) idx += s_end[wv][idx + bit - 1] <= eb ? (int)bit : 0;
    unsigned long long run = 0;
    for (int q = 0; q < 8; ++q) {
      const uint64_t e = eb + q;
      const uint32_t c = (uint32_t)(word >> (8 * q)) & 0xffu;
      const bool sv = e >= e0 && e < e1 && hp_dsurv(c, H);
      while (idx < 64 && s_end[wv][idx] <= e) {  // the entry starts a later row: flush the run
        if (run) atomicAdd(&s_acc[wv][idx], run);
        run = 0;
        ++idx;
      }
      if (!sv) continue;
      ++tc;
      const unsigned long long add = (1ull << 40) | c;
      if (e < last_end) {
        run += add;
      } else {  // more than 64 rows in this tile: search the offsets
        uint64_t a = r0, b = nU;
        while (b - a > 1) {
          const uint64_t md = (a + b) >> 1;
          if (g.off[ua + md] <= e) a = md; else b = md;
        }
        atomicAdd(&wu[a], add);
      }
    }
    if (run && idx < 64) atomicAdd(&s_acc[wv][idx], run);
    tc = (uint32_t)wave_sum((uint64_t)tc);
    if (lane == 0) tcnt[tile - t0] = tc;
    wave_sync_lds();
    const unsigned long long v = s_acc[wv][lane];
    if (v) {
      atomicAdd(&wu[rl], v);
      s_acc[wv][lane] = 0;
    }
    wave_sync_lds();
  }
}

__global__ void k_hp_unpack(unsigned long long* __restrict__ wu, uint32_t* __restrict__ cnt, uint64_t nU) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nU; r += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long x = wu[r];
    cnt[r] = (uint32_t)(x >> 40);
    wu[r] = x & ((1ull << 40) - 1);
  }
}

// Per graph, one pass over the adjacency entries e = (u -> v): the degree class
// of v (dcls[e] = min(deg v, 255): path 4 filters N(u) by it, coalesced bytes
// instead of a degree gather), deg v itself (kd, when given: the count-metric
// row kernels carry it) and, for deg v <= 254, the entries of N(v) at or below
// u (drank, when given: its rank there -- the survivor lists' fill reads it
// instead of searching N(v) on every call).  deg v comes from off[v], off[v + 1]
// (one line, which the search of N(v) needs anyway), a lane's HP_WR gathers in
// flight together.  Edge-parallel over HP_WTILE-entry tiles, each entry's row
// from its tile's first row by a search of 64 row ends held in lanes.  C4:
// 200 ms, against 68 + 178 ms for round 5's degree-gather and binary-search
// passes; an 8-way split search (7 pivot loads a round) measured slower here
// (312 ms fused, 374 ms in two passes): the lists are at most 254 entries, so
// the binary search's later probes hit lines already fetched.
__global__ __launch_bounds__(NT) void k_hp_entry_classes(const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ keys, uint64_t S, uint64_t M,
                                                         const uint32_t* __restrict__ tile_row,
                                                         uint8_t* __restrict__ dcls, uint32_t* __restrict__ kd,
                                                         uint8_t* __restrict__ drank) {
  const int lane = lane_id(), wv = wave_id();
  const uint64_t nt = (M + HP_WTILE - 1) / HP_WTILE;
  for (uint64_t tile = (uint64_t)blockIdx.x * NWAVE + wv; tile < nt; tile += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t base = tile * HP_WTILE;
    const uint64_t r0 = tile_row[tile];
    const uint64_t rl = r0 + lane;
    const uint64_t rend = rl < S ? off[rl + 1] : ~0ull;
    const uint64_t last_end = __shfl(rend, 63, 64);
    // the lane's HP_WR entries: keys (coalesced), then their row bounds all in flight together
    uint32_t v[HP_WR];
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      v[i] = e < M ? keys[e] : 0u;
    }
    uint64_t o[HP_WR], o1[HP_WR];
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      o[i] = off[v[i]];
      o1[i] = off[v[i] + 1];
    }
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      const uint64_t d64 = o1[i] - o[i];
      const uint32_t d = d64 > 0xffffffffull ? 0xffffffffu : (uint32_t)d64;
      if (e < M) {
        dcls[e] = (uint8_t)(d < 255u ? d : 255u);
        if (kd) kd[e] = d;
      }
    }
    if (!drank) continue;
#pragma unroll 1
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      int lo = 0, hi = 64;
      while (lo < hi) {
        const int md = (lo + hi) >> 1;
        const uint64_t x = __shfl(rend, md, 64);
        if (x <= e) lo = md + 1; else hi = md;
      }
      if (e >= M) continue;
      const uint64_t d = o1[i] - o[i];
      if (d == 0 || d > HP_DCLS_MAX) {
        drank[e] = 0;
        continue;
      }
      uint64_t r = r0 + lo;
      if (e >= last_end) {
        uint64_t a = r0, b = S;
        while (b - a > 1) {
          const uint64_t md = (a + b) >> 1;
          if (off[md] <= e) a = md; else b = md;
        }
        r = a;
      }
      drank[e] = (uint8_t)upper_bound_u32(keys + o[i], (uint32_t)d, (uint32_t)r);
    }
  }
}

// (v << 32 | u) for every entry u -> v, in CSR order (the transposed build's
// sort input): edge-parallel over HP_WTILE-entry tiles, each entry's row from
// its tile's first row (tile_row) by a search of 64 row ends held in lanes
// (a binary search of all offsets per entry cost ~85 ms on C4).
__global__ __launch_bounds__(NT) void k_transpose_keys(const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                                                       uint64_t S, uint64_t M, const uint32_t* __restrict__ tile_row,
                                                       uint64_t* __restrict__ out) {
  const int lane = lane_id(), wv = wave_id();
  const uint64_t nt = (M + HP_WTILE - 1) / HP_WTILE;
  for (uint64_t tile = (uint64_t)blockIdx.x * NWAVE + wv; tile < nt; tile += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t base = tile * HP_WTILE;
    const uint64_t r0 = tile_row[tile];
    const uint64_t rl = r0 + lane;
    const uint64_t rend = rl < S ? off[rl + 1] : ~0ull;
    const uint64_t last_end = __shfl(rend, 63, 64);
#pragma unroll 1
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      const uint32_t w = e < M ? keys[e] : 0u;
      int lo = 0, hi = 64;
      while (lo < hi) {
        const int md = (lo + hi) >> 1;
        const uint64_t x = __shfl(rend, md, 64);
        if (x <= e) lo = md + 1; else hi = md;
      }
      if (e >= M) continue;
      uint64_t r = r0 + lo;
      if (e >= last_end) {
        uint64_t a = r0, b = S;
        while (b - a > 1) {
          const uint64_t md = (a + b) >> 1;
          if (off[md] <= e) a = md; else b = md;
        }
        r = a;
      }
      out[e] = ((uint64_t)w << 32) | r;
    }
  }
}

// ---------------------------------------------------------------- membership table build (per graph)
// The table's size bound: the entries w > u, sum over rows of deg u - xs[u]
// (xs = the entries at or below u, k_hp_xs) -- a streaming read of two S-word
// arrays instead of a pass over the adjacency with a wave per row.
__global__ void k_etab_upper(const uint32_t* __restrict__ deg, const uint32_t* __restrict__ xs, uint64_t S,
                             unsigned long long* __restrict__ count) {
  uint64_t c = 0;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < S; u += (uint64_t)gridDim.x * blockDim.x)
    c += deg[u] - xs[u];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane_id() == 0 && c) atomicAdd(count, (unsigned long long)c);
}

// Insert one key: the bucket line is read whole (8 slots, one round trip),
// then its first empty slot is claimed by one CAS; a lost race re-reads the
// same bucket.  Slots only go from empty to full and a writer claims only the
// first empty slot it saw, so a bucket never has a hole and a key never lands
// twice -- et_has's rule (absent once a bucket with an empty slot lacks it)
// holds.
// (from bucket b on: the probe of a key whose home bucket was found full)
__device__ __forceinline__ void et_insert_at(uint64_t* __restrict__ tab, uint32_t bits, uint64_t key, uint64_t b) {
  const uint64_t mask = (1ull << bits) - 1;
  for (uint64_t probe = 0; probe <= mask;) {
    unsigned long long* q = (unsigned long long*)(tab + b * ET_SLOTS);
    uint64_t s[ET_SLOTS];
#pragma unroll
    for (int j = 0; j < ET_SLOTS; ++j) s[j] = __hip_atomic_load(q + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int first = -1;
    bool hit = false;
#pragma unroll
    for (int j = ET_SLOTS - 1; j >= 0; --j) {
      hit |= s[j] == key;
      if (s[j] == ET_EMPTY) first = j;
    }
    if (hit) return;
    if (first < 0) {
      b = (b + 1) & mask;
      ++probe;
      continue;
    }
    const unsigned long long cur = atomicCAS(q + first, ET_EMPTY, (unsigned long long)key);
    if (cur == ET_EMPTY || cur == key) return;
  }
}

// N keys at once, two round trips for all of them instead of two each: their
// home buckets are read together with plain loads (a hint: a stale line only
// lacks keys, never shows a slot full that is empty), then each claims the
// first empty slot it saw by CAS, the N CASes issued together.  A CAS that
// finds another key moves to the next slot (the CAS's answer is the truth, so
// no re-read); a bucket seen full probes on from the next bucket (et_insert_at).
// A writer claims slot j only after finding slots below j full and stops at
// its own key, so buckets keep no holes and no key lands twice.
template <int N>
__device__ __forceinline__ void et_insert_n(uint64_t* __restrict__ tab, uint32_t bits, const uint64_t (&key)[N],
                                            const bool (&act)[N]) {
  const uint64_t mask = (1ull << bits) - 1;
  ulonglong2 q[N][4];
  uint64_t b[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    b[i] = et_mix(key[i]) >> (64 - bits);
    const ulonglong2* p = (const ulonglong2*)(tab + (act[i] ? b[i] : 0ull) * ET_SLOTS);
#pragma unroll
    for (int j = 0; j < 4; ++j) q[i][j] = act[i] ? p[j] : make_ulonglong2(0, 0);
  }
  int pos[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t sl[ET_SLOTS] = {q[i][0].x, q[i][0].y, q[i][1].x, q[i][1].y,
                                   q[i][2].x, q[i][2].y, q[i][3].x, q[i][3].y};
    int first = ET_SLOTS;
    bool hit = false;
#pragma unroll
    for (int j = ET_SLOTS - 1; j >= 0; --j) {
      hit |= sl[j] == key[i];
      if (sl[j] == ET_EMPTY) first = j;
    }
    pos[i] = !act[i] || hit ? -1 : first;  // ET_SLOTS: the bucket is full
  }
  unsigned long long cur[N];
#pragma unroll
  for (int i = 0; i < N; ++i)
    cur[i] = pos[i] >= 0 && pos[i] < ET_SLOTS
                 ? atomicCAS((unsigned long long*)(tab + b[i] * ET_SLOTS + pos[i]), ET_EMPTY,
                             (unsigned long long)key[i])
                 : ET_EMPTY;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (pos[i] < 0) continue;
    int j = pos[i];
    if (j < ET_SLOTS) {
      unsigned long long c = cur[i];
      while (c != ET_EMPTY && c != key[i] && ++j < ET_SLOTS)
        c = atomicCAS((unsigned long long*)(tab + b[i] * ET_SLOTS + j), ET_EMPTY, (unsigned long long)key[i]);
    }
    if (j >= ET_SLOTS) et_insert_at(tab, bits, key[i], (b[i] + 1) & mask);
  }
}

// The entries w > u inserted edge-parallel: a wave takes HP_WTILE consecutive
// adjacency entries (coalesced keys, every lane busy whatever the degrees),
// finding each entry's row from the tile's first row like k_hp_drank; a
// lane's HP_WR keys go in together (et_insert_n).
__global__ __launch_bounds__(NT) void k_etab_insert(const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                                                    uint64_t S, uint64_t M, const uint32_t* __restrict__ tile_row,
                                                    uint64_t* __restrict__ tab, uint32_t bits) {
  const int lane = lane_id(), wv = wave_id();
  const uint64_t nt = (M + HP_WTILE - 1) / HP_WTILE;
  for (uint64_t tile = (uint64_t)blockIdx.x * NWAVE + wv; tile < nt; tile += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t base = tile * HP_WTILE;
    const uint64_t r0 = tile_row[tile];
    const uint64_t rl = r0 + lane;
    const uint64_t rend = rl < S ? off[rl + 1] : ~0ull;
    const uint64_t last_end = __shfl(rend, 63, 64);
    uint64_t key[HP_WR];
    bool act[HP_WR];
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      const uint32_t w = e < M ? keys[e] : 0u;
      int lo = 0, hi = 64;
      while (lo < hi) {
        const int md = (lo + hi) >> 1;
        const uint64_t x = __shfl(rend, md, 64);
        if (x <= e) lo = md + 1; else hi = md;
      }
      uint64_t r = r0 + lo;
      if (e < M && e >= last_end) {
        uint64_t a = r0, b = S;
        while (b - a > 1) {
          const uint64_t md = (a + b) >> 1;
          if (off[md] <= e) a = md; else b = md;
        }
        r = a;
      }
      act[i] = e < M && w > r;
      key[i] = (r << 32) | w;
    }
    et_insert_n<HP_WR>(tab, bits, key, act);
  }
}

// (sdo: also the entry packed for the row batches, deg v << 48 | n << 40 | o,
// where [o, o + n) is the part of N(v) above the entry's row u -- found here
// by a binary search of v's short list (deg v <= 254) -- so that the batches
// enumerate only the wedges w > u and skip the gather of v's row bounds; and
// W+(u) = the sum of n over S(u), accumulated into wu (zeroed by the caller):
// a tighter bound than W(u) for the bins, the tables and the batch budget)
__global__ __launch_bounds__(NT) void k_hp_dcls_fill(GraphView g, const uint8_t* __restrict__ dcls, uint32_t H,
                                                     uint64_t ua, uint64_t nU, uint64_t e0, uint64_t e1,
                                                     const uint32_t* __restrict__ tile_row,
                                                     const uint64_t* __restrict__ tpre, uint32_t* __restrict__ skeys,
                                                     uint64_t* __restrict__ sdo, unsigned long long* __restrict__ wu,
                                                     const uint8_t* __restrict__ drank) {
  __shared__ unsigned long long s_acc[NWAVE][64];
  const int lane = lane_id(), wv = wave_id();
  const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE;
  s_acc[wv][lane] = 0;
  for (uint64_t tile = t0 + (uint64_t)blockIdx.x * NWAVE + wv; tile < t1; tile += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t base = tile * HP_WTILE;
    uint64_t pos = tpre[tile - t0];
    const uint64_t tr = tile_row[tile];
    const uint64_t r0 = tr > ua ? tr - ua : 0;  // first row of the tile inside the range
    const uint64_t rl = r0 + lane;
    const uint64_t rend = rl < nU ? g.off[ua + rl + 1] : ~0ull;
    const uint64_t last_end = __shfl(rend, 63, 64);
    uint32_t c[HP_WR];
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      c[i] = e >= e0 && e < e1 ? (uint32_t)dcls[e] : 0u;
    }
#pragma unroll
    for (int i = 0; i < HP_WR; ++i) {
      const uint64_t e = base + (uint64_t)i * 64 + lane;
      const bool sv = hp_dsurv(c[i], H);
      const uint64_t m = __ballot(sv);
      if (m) {
        int lo = 0, hi = 64;  // local row of e
        while (lo < hi) {
          const int md = (lo + hi) >> 1;
          const uint64_t x = __shfl(rend, md, 64);
          if (x <= e) lo = md + 1; else hi = md;
        }
        if (sv) {
          const uint64_t q = pos + (uint64_t)__popcll(m & ((1ull << lane) - 1));
          const uint32_t v = g.keys[e];
          skeys[q] = v;
          if (sdo) {
            uint64_t r = r0 + lo;
            if (e >= last_end) {  // more than 64 rows in this tile: search the offsets
              uint64_t a = r0, b = nU;
              while (b - a > 1) {
                const uint64_t md = (a + b) >> 1;
                if (g.off[ua + md] <= e) a = md; else b = md;
              }
              r = a;
            }
            const uint32_t u = (uint32_t)(ua + r);
            const uint64_t o = g.off[v];
            uint32_t l = 0;  // the first entry of N(v) above u
            if (drank) {
              l = drank[e];
            } else if (c[i] <= 16) {  // short lists: count the entries <= u with independent loads (one round trip)
              uint32_t kk[16];
#pragma unroll
              for (int q = 0; q < 16; ++q) kk[q] = (uint32_t)q < c[i] ? g.keys[o + q] : 0xffffffffu;
#pragma unroll
              for (int q = 0; q < 16; ++q) l += kk[q] <= u ? 1u : 0u;
            } else {
              uint32_t h = c[i];
              while (l < h) {
                const uint32_t md = (l + h) >> 1;
                if (g.keys[o + md] <= u) l = md + 1; else h = md;
              }
            }
            const uint32_t n = c[i] - l;
            sdo[q] = (uint64_t)c[i] << 48 | (uint64_t)n << HP_SDO_SH | (o + l);
            if (n) {
              if (e < last_end) atomicAdd(&s_acc[wv][lo], (unsigned long long)n);
              else atomicAdd(&wu[r], (unsigned long long)n);
            }
          }
        }
      }
      pos += (uint64_t)__popcll(m);
    }
    if (sdo) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      const unsigned long long x = s_acc[wv][lane];
      if (x) {
        atomicAdd(&wu[rl], x);
        s_acc[wv][lane] = 0;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
  }
}

// k_hp_dcls_fill with eight consecutive entries per lane (the layout of
// k_hp_dcls_rows8): one 8-byte load of classes and of ranks, the lane's
// survivors placed at a wave scan of the per-lane counts, the row of the
// lane's first entry found once and walked forward.  Needs sdo and drank.
__global__ __launch_bounds__(NT) void k_hp_dcls_fill8(GraphView g, const uint8_t* __restrict__ dcls, uint32_t H,
                                                      uint64_t ua, uint64_t nU, uint64_t e0, uint64_t e1,
                                                      const uint32_t* __restrict__ tile_row,
                                                      const uint64_t* __restrict__ tpre, uint32_t* __restrict__ skeys,
                                                      uint64_t* __restrict__ sdo, unsigned long long* __restrict__ wu,
                                                      const uint8_t* __restrict__ drank) {
  __shared__ unsigned long long s_acc[NWAVE][64];
  __shared__ uint64_t s_end[NWAVE][64];
  const int lane = lane_id(), wv = wave_id();
  const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE;
  s_acc[wv][lane] = 0;
  for (uint64_t tile = t0 + (uint64_t)blockIdx.x * NWAVE + wv; tile < t1; tile += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t base = tile * HP_WTILE;
    const uint64_t tr = tile_row[tile];
    const uint64_t r0 = tr > ua ? tr - ua : 0;
    const uint64_t rl = r0 + lane;
    s_end[wv][lane] = rl < nU ? g.off[ua + rl + 1] : ~0ull;
    wave_sync_lds();
    const uint64_t last_end = s_end[wv][63];
    const uint64_t eb = base + (uint64_t)lane * 8;
    uint64_t word = 0, rk = 0;
    if (eb + 8 <= e1 && eb >= e0) {
      word = *(const uint64_t*)(dcls + eb);
      rk = *(const uint64_t*)(drank + eb);
    } else {
      for (int q = 0; q < 8; ++q)
        if (eb + q >= e0 && eb + q < e1) {
          word |= (uint64_t)dcls[eb + q] << (8 * q);
          rk |= (uint64_t)drank[eb + q] << (8 * q);
        }
    }
    uint32_t mine = 0;  // survivors among this lane's entries (in range)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint64_t e = eb + q;
      mine += (e >= e0 && e < e1 && hp_dsurv((uint32_t)(word >> (8 * q)) & 0xffu, H)) ? 1u : 0u;
    }
    uint64_t pos = tpre[tile - t0] + wave_incl_scan((uint64_t)mine) - mine;
    int idx = 0;
#pragma unroll
    for (uint32_t bit = 32; bit > 0; bit >>= 1) idx += s_end[wv][idx + bit - 1] <= eb ? (int)bit : 0;
    unsigned long long run = 0;
    for (int q = 0; q < 8; ++q) {
      const uint64_t e = eb + q;
      const uint32_t c = (uint32_t)(word >> (8 * q)) & 0xffu;
      while (idx < 64 && s_end[wv][idx] <= e) {
        if (run) atomicAdd(&s_acc[wv][idx], run);
        run = 0;
        ++idx;
      }
      if (!(e >= e0 && e < e1 && hp_dsurv(c, H))) continue;
      uint64_t r = r0 + (uint64_t)idx;
      if (e >= last_end) {
        uint64_t a = r0, b = nU;
        while (b - a > 1) {
          const uint64_t md = (a + b) >> 1;
          if (g.off[ua + md] <= e) a = md; else b = md;
        }
        r = a;
      }
      const uint32_t v = g.keys[e];
      const uint32_t l = (uint32_t)(rk >> (8 * q)) & 0xffu;
      const uint64_t o = g.off[v];
      const uint32_t n = c - l;
      skeys[pos] = v;
      sdo[pos] = (uint64_t)c << 48 | (uint64_t)n << HP_SDO_SH | (o + l);
      ++pos;
      if (n) {
        if (e < last_end) run += n;
        else atomicAdd(&wu[r], (unsigned long long)n);
      }
    }
    if (run && idx < 64) atomicAdd(&s_acc[wv][idx], run);
    wave_sync_lds();
    const unsigned long long x = s_acc[wv][lane];
    if (x) {
      atomicAdd(&wu[rl], x);
      s_acc[wv][lane] = 0;
    }
    wave_sync_lds();
  }
}

// ---------------------------------------------------------------- survivor lists in three streaming kernels
// A one-pass build (classes, look-back, then per survivor its key and off[v],
// three workgroups per CU at 163 VGPRs) waited on five dependent round trips
// per tile (C4 H=16: 4.6e7 survivors among 3.5e9 entries, 7.2 ms; removed in
// round 5).  Here the chain is cut where the parallelism changes:
//   k_dc_count   a wave per 512-entry wave tile: its survivors counted (one
//                8-byte class word per lane); the counts are scanned;
//   k_dc_place   the same tiles again: each survivor's entry e and row r
//                (row ends of the tile's first 64 rows in LDS, as the fill) at
//                its position in entry order;
//   k_dc_gather  a thread per survivor: key v = keys[e], class, rank, off[v] --
//                independent across survivors, thousands in flight per CU --
//                the packed entry, and (count << 40 | W+) per row by one
//                atomic per run of equal rows in a wave.
__device__ __forceinline__ uint32_t hp_dword(const uint8_t* __restrict__ dcls, uint64_t eb, uint64_t e0, uint64_t e1,
                                             uint64_t* w) {
  uint64_t x = 0;
  if (eb >= e0 && eb + 8 <= e1) x = *(const uint64_t*)(dcls + eb);
  else
    for (int q = 0; q < 8; ++q)
      if (eb + q >= e0 && eb + q < e1) x |= (uint64_t)dcls[eb + q] << (8 * q);
  *w = x;
  return 0;
}

__device__ __forceinline__ uint32_t hp_dsurv8(uint64_t word, uint32_t H) {
  uint32_t m = 0;  // bit q: byte q is a survivor class
#pragma unroll
  for (int q = 0; q < 8; ++q) m |= hp_dsurv((uint32_t)(word >> (8 * q)) & 0xffu, H) ? 1u << q : 0u;
  return m;
}

// smask[(wt - t0) * 64 + lane]: bit q = entry wt * 512 + 8 lane + q survives
// (k_dc_place reads these 64 bytes per wave tile instead of its 512 class bytes)
__global__ __launch_bounds__(NT) void k_dc_count(const uint8_t* __restrict__ dcls, uint32_t H, uint64_t e0, uint64_t e1,
                                                 uint32_t* __restrict__ tcn, uint8_t* __restrict__ smask) {
  const int lane = lane_id();
  const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE;
  for (uint64_t wt = t0 + (uint64_t)blockIdx.x * NWAVE + wave_id(); wt < t1; wt += (uint64_t)gridDim.x * NWAVE) {
    uint64_t word;
    hp_dword(dcls, wt * HP_WTILE + (uint64_t)lane * 8, e0, e1, &word);
    const uint32_t m = hp_dsurv8(word, H);
    smask[(wt - t0) * 64 + lane] = (uint8_t)m;
    const uint64_t c = wave_sum((uint64_t)__popc(m));
    if (lane == 0) tcn[wt - t0] = (uint32_t)c;
  }
}

__global__ __launch_bounds__(NT) void k_dc_place(GraphView g, const uint8_t* __restrict__ smask,
                                                 uint64_t ua, uint64_t nU, uint64_t e0, uint64_t e1,
                                                 const uint32_t* __restrict__ tile_row,
                                                 const uint64_t* __restrict__ tpre, uint64_t* __restrict__ se,
                                                 uint32_t* __restrict__ sr) {
  __shared__ uint64_t s_end[NWAVE][64];
  const int lane = lane_id(), wv = wave_id();
  const uint64_t t0 = e0 / HP_WTILE, t1 = (e1 + HP_WTILE - 1) / HP_WTILE;
  for (uint64_t wt = t0 + (uint64_t)blockIdx.x * NWAVE + wv; wt < t1; wt += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t eb = wt * HP_WTILE + (uint64_t)lane * 8;
    uint32_t m = smask[(wt - t0) * 64 + lane];
    if (__ballot(m != 0) == 0) continue;  // no survivor in the wave tile: no row ends needed
    const uint64_t tr = tile_row[wt];
    const uint64_t r0 = tr > ua ? tr - ua : 0;
    const uint64_t rl = r0 + lane;
    s_end[wv][lane] = rl < nU ? g.off[ua + rl + 1] : ~0ull;
    wave_sync_lds();
    const uint32_t mine = (uint32_t)__popc(m);
    uint64_t pos = tpre[wt - t0] + wave_incl_scan((uint64_t)mine) - mine;
    int idx = 0;  // rows of the wave tile ending at or before this lane's first entry
#pragma unroll
    for (uint32_t bit = 32; bit > 0; bit >>= 1) idx += s_end[wv][idx + bit - 1] <= eb ? (int)bit : 0;
    while (m) {
      const int q = __builtin_ctz(m);
      m &= m - 1;
      const uint64_t e = eb + q;
      while (idx < 64 && s_end[wv][idx] <= e) ++idx;
      uint64_t r = r0 + (uint64_t)idx;
      if (idx >= 64) {  // beyond the tile's first 64 rows: search the range's row ends
        uint64_t lo = r0, hi = nU;
        while (hi - lo > 1) {
          const uint64_t md = (lo + hi) >> 1;
          if (g.off[ua + md] <= e) lo = md; else hi = md;
        }
        r = lo;
      }
      se[pos] = e;
      sr[pos] = (uint32_t)r;
      ++pos;
    }
    wave_sync_lds();
  }
}

__global__ __launch_bounds__(NT) void k_dc_gather(GraphView g, const uint8_t* __restrict__ dcls,
                                                  const uint8_t* __restrict__ drank, const uint64_t* __restrict__ se,
                                                  const uint32_t* __restrict__ sr, uint64_t ns,
                                                  uint32_t* __restrict__ skeys, uint64_t* __restrict__ sdo,
                                                  unsigned long long* __restrict__ wu) {
  const int lane = lane_id();
  for (uint64_t b = (uint64_t)blockIdx.x * NT; b < ns; b += (uint64_t)gridDim.x * NT) {  // uniform per wave
    const uint64_t i = b + threadIdx.x;
    const bool ok = i < ns;
    uint32_t r = 0xffffffffu;
    unsigned long long x = 0;
    if (ok) {
      const uint64_t e = se[i];
      r = sr[i];
      const uint32_t c = dcls[e], l = drank[e];
      const uint32_t v = g.keys[e];
      const uint64_t o = g.off[v];
      const uint32_t n = c - l;  // the part of N(v) above the row
      skeys[i] = v;
      sdo[i] = (uint64_t)c << 48 | (uint64_t)n << HP_SDO_SH | (o + l);
      x = (1ull << 40) | n;
    }
    // rows are non-decreasing over consecutive survivors: a segmented sum per run, one atomic at its end
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d, 64);
      const uint32_t ry = __shfl_up(r, d, 64);
      if (lane >= d && ry == r) x += y;
    }
    const uint32_t rn = __shfl_down(r, 1, 64);
    if (ok && (lane == 63 || rn != r)) atomicAdd(&wu[r], x);
  }
}

// ---------------------------------------------------------------- class-ordered short lists (per graph)
// The count metrics do not depend on the order of S(u).  So the graph keeps,
// per row, its short entries -- v with 1 <= deg v <= HP_DCLS_MAX, packed as
// the survivor lists are (key v, deg v << 48 | n << 40 | o) -- ordered by
// deg v: S(u) for any H up to the classes kept is a prefix of the row's list,
// and a call only measures the prefixes (k_sl_rows: a search of each row's
// classes, W+(u) from the per-graph prefix of n) instead of compacting the
// range's classes and gathering off[v] per survivor.  Built once in
// nlp_graph_create from the degree-class compaction at the classes kept
// (k_dc_*), then k_sl_sort (which also writes the prefix of n).

// k_sl_sort: a wave per row, stable by class, and pn[i] = the inclusive prefix
// of n over the row's sorted list.  Rows of at most 64 entries rank every lane
// against every other (the prefix: a wave scan of n in sorted order through
// LDS); longer rows count their classes in an LDS histogram, scan it, and
// place 64 entries per step ranked by a ballot multisplit on the class (cursor
// advanced by the last lane of each class), then scan the row just written
// (cache-warm; round 5 ran the prefix as a separate pass: 31 ms on C4), each
// of those loops with several steps' loads in flight.  Rows of long_min
// entries or more are listed for k_sl_sort_long instead (one wave would walk
// a hub's ~1e6 entries alone).
__global__ __launch_bounds__(NT) void k_sl_sort(const uint64_t* __restrict__ lo, uint64_t S,
                                                const uint32_t* __restrict__ ikeys, const uint64_t* __restrict__ isdo,
                                                uint32_t* __restrict__ okeys, uint64_t* __restrict__ osdo,
                                                uint8_t* __restrict__ ocls, uint32_t* __restrict__ pn,
                                                uint64_t long_min, uint32_t* __restrict__ longrows,
                                                uint32_t* __restrict__ nlong) {
  __shared__ uint32_t s_h[NWAVE][256];
  __shared__ uint32_t s_n[NWAVE][64];
  const int lane = lane_id(), wv = wave_id();
  for (uint64_t u = (uint64_t)blockIdx.x * NWAVE + wv; u < S; u += (uint64_t)gridDim.x * NWAVE) {
    const uint64_t s = lo[u], n = lo[u + 1] - s;
    if (n == 0) continue;
    if (n >= long_min) {  // a hub's list: a workgroup of its own (k_sl_sort_long)
      if (lane == 0) longrows[atomicAdd(nlong, 1u)] = (uint32_t)u;
      continue;
    }
    if (n <= 64) {
      const bool ok = (uint64_t)lane < n;
      const uint64_t sd = ok ? isdo[s + lane] : 0ull;
      const uint32_t key = ok ? ikeys[s + lane] : 0u;
      const uint32_t c = ok ? (uint32_t)(sd >> 48) : 0xffffu;
      uint32_t rank = 0;
      for (int j = 0; j < (int)n; ++j) {
        const uint32_t cj = __shfl(c, j, 64);
        rank += (cj < c || (cj == c && j < lane)) ? 1u : 0u;
      }
      if (ok) {
        okeys[s + rank] = key;
        osdo[s + rank] = sd;
        ocls[s + rank] = (uint8_t)c;
        s_n[wv][rank] = (uint32_t)(sd >> HP_SDO_SH) & 0xffu;
      }
      wave_sync_lds();
      const uint64_t incl = wave_incl_scan(ok ? (uint64_t)s_n[wv][lane] : 0ull);
      if (ok) pn[s + lane] = (uint32_t)incl;
      wave_sync_lds();
      continue;
    }
    // a long row (a hub's short list can hold ~1e6 entries, and one wave owns
    // it): every loop below issues SL_U steps of loads before using them
    constexpr int SL_U = 8;
    for (int q = lane; q < 256; q += 64) s_h[wv][q] = 0;
    wave_sync_lds();
    for (uint64_t j0 = 0; j0 < n; j0 += 64 * SL_U) {
      uint32_t cq[SL_U];
#pragma unroll
      for (int q = 0; q < SL_U; ++q) {
        const uint64_t j = j0 + (uint64_t)q * 64 + lane;
        cq[q] = j < n ? (uint32_t)(isdo[s + j] >> 48) & 255u : 256u;
      }
#pragma unroll
      for (int q = 0; q < SL_U; ++q)
        if (cq[q] < 256u) atomicAdd(&s_h[wv][cq[q]], 1u);
    }
    wave_sync_lds();
    {
      uint32_t h[4], t = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        h[q] = s_h[wv][4 * lane + q];
        t += h[q];
      }
      uint32_t ex = (uint32_t)wave_incl_scan((uint64_t)t) - t;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s_h[wv][4 * lane + q] = ex;
        ex += h[q];
      }
    }
    wave_sync_lds();
    constexpr int SL_P = 4;
    for (uint64_t j00 = 0; j00 < n; j00 += 64 * SL_P) {
      uint64_t sdq[SL_P];
      uint32_t kq[SL_P];
#pragma unroll
      for (int q = 0; q < SL_P; ++q) {
        const uint64_t j = j00 + (uint64_t)q * 64 + lane;
        sdq[q] = j < n ? isdo[s + j] : 0ull;
        kq[q] = j < n ? ikeys[s + j] : 0u;
      }
#pragma unroll
      for (int q = 0; q < SL_P; ++q) {
        const uint64_t j = j00 + (uint64_t)q * 64 + lane;
        if (j00 + (uint64_t)q * 64 >= n) break;  // wave-uniform
        const bool ok = j < n;
        const uint64_t sd = sdq[q];
        const uint32_t c = (uint32_t)(sd >> 48) & 255u;
        uint64_t m = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const bool bit = (c >> b) & 1u;
          const uint64_t bb = __ballot(bit);
          m &= bit ? bb : ~bb;
        }
        const uint32_t base = s_h[wv][c];
        wave_sync_lds();
        if (ok) {
          const uint64_t p = s + base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
          okeys[p] = kq[q];
          osdo[p] = sd;
          ocls[p] = (uint8_t)c;
          if ((m >> lane) == 1ull) s_h[wv][c] = base + (uint32_t)__popcll(m);  // the class's last lane
        }
        wave_sync_lds();
      }
    }
    // the row's prefix of n, read back from the list just written by this wave
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    uint64_t carry = 0;
    for (uint64_t j0 = 0; j0 < n; j0 += 64 * SL_U) {
      uint64_t xq[SL_U];
#pragma unroll
      for (int q = 0; q < SL_U; ++q) {
        const uint64_t j = j0 + (uint64_t)q * 64 + lane;
        xq[q] = j < n ? (osdo[s + j] >> HP_SDO_SH) & 0xffull : 0ull;
      }
#pragma unroll
      for (int q = 0; q < SL_U; ++q) {
        const uint64_t j = j0 + (uint64_t)q * 64 + lane;
        const uint64_t incl = wave_incl_scan(xq[q]) + carry;
        if (j < n) pn[s + j] = (uint32_t)incl;
        carry = __shfl(incl, 63, 64);
      }
    }
  }
}

// k_sl_sort_long: the listed long rows, a workgroup of SLL_NW waves each,
// every wave a contiguous chunk of the row: per-wave class histograms, per
// class the waves' exclusive offsets after the classes' starts (stable: chunk
// order is row order), every chunk placed by the same ballot multisplit, then
// the prefix of n as chunk sums, their exclusive scan, and a scan per chunk.
constexpr int SLL_NW = 16, SLL_NT = 64 * SLL_NW;
constexpr uint64_t SL_LONG = 4096;  // short entries from which a row is k_sl_sort_long's
__global__ __launch_bounds__(SLL_NT) void k_sl_sort_long(const uint64_t* __restrict__ lo,
                                                         const uint32_t* __restrict__ rows, uint32_t nrows,
                                                         const uint32_t* __restrict__ ikeys,
                                                         const uint64_t* __restrict__ isdo,
                                                         uint32_t* __restrict__ okeys, uint64_t* __restrict__ osdo,
                                                         uint8_t* __restrict__ ocls, uint32_t* __restrict__ pn) {
  __shared__ uint32_t s_h[SLL_NW][256];
  __shared__ uint64_t s_w4[4];
  __shared__ uint64_t s_sum[SLL_NW];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  constexpr int U = 8, P = 4;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t u = rows[r];
    const uint64_t s = lo[u], n = lo[u + 1] - s;
    const uint64_t chunk = ((n + SLL_NW - 1) / SLL_NW + 63) / 64 * 64;
    const uint64_t c0 = min(n, (uint64_t)wv * chunk), c1 = min(n, c0 + chunk);
    for (int q = lane; q < 256; q += 64) s_h[wv][q] = 0;
    wave_sync_lds();
    for (uint64_t j0 = c0; j0 < c1; j0 += 64 * U) {
      uint32_t cq[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const uint64_t j = j0 + (uint64_t)q * 64 + lane;
        cq[q] = j < c1 ? (uint32_t)(isdo[s + j] >> 48) & 255u : 256u;
      }
#pragma unroll
      for (int q = 0; q < U; ++q)
        if (cq[q] < 256u) atomicAdd(&s_h[wv][cq[q]], 1u);
    }
    __syncthreads();
    uint32_t run = 0;
    if (t < 256) {
      for (int w = 0; w < SLL_NW; ++w) {
        const uint32_t c = s_h[w][t];
        s_h[w][t] = run;
        run += c;
      }
    }
    uint64_t incl = 0;
    if (t < 256) {  // waves 0-3: the classes' starts
      incl = wave_incl_scan((uint64_t)run);
      if (lane == 63) s_w4[wv] = incl;
    }
    __syncthreads();
    if (t < 256) {
      uint64_t pre = 0;
      for (int w = 0; w < wv; ++w) pre += s_w4[w];
      const uint32_t cs = (uint32_t)(pre + incl - run);
      for (int w = 0; w < SLL_NW; ++w) s_h[w][t] += cs;
    }
    __syncthreads();
    for (uint64_t j00 = c0; j00 < c1; j00 += 64 * P) {
      uint64_t sdq[P];
      uint32_t kq[P];
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const uint64_t j = j00 + (uint64_t)q * 64 + lane;
        sdq[q] = j < c1 ? isdo[s + j] : 0ull;
        kq[q] = j < c1 ? ikeys[s + j] : 0u;
      }
#pragma unroll
      for (int q = 0; q < P; ++q) {
        if (j00 + (uint64_t)q * 64 >= c1) break;  // wave-uniform
        const uint64_t j = j00 + (uint64_t)q * 64 + lane;
        const bool ok = j < c1;
        const uint32_t c = (uint32_t)(sdq[q] >> 48) & 255u;
        uint64_t m = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const bool bit = (c >> b) & 1u;
          const uint64_t bb = __ballot(bit);
          m &= bit ? bb : ~bb;
        }
        const uint32_t base = s_h[wv][c];
        wave_sync_lds();
        if (ok) {
          const uint64_t p = s + base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
          okeys[p] = kq[q];
          osdo[p] = sdq[q];
          ocls[p] = (uint8_t)c;
          if ((m >> lane) == 1ull) s_h[wv][c] = base + (uint32_t)__popcll(m);
        }
        wave_sync_lds();
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // the prefix of n over the sorted row: chunk sums, their exclusive scan, a scan per chunk
    uint64_t sum = 0;
    for (uint64_t j0 = c0; j0 < c1; j0 += 64 * U) {
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const uint64_t j = j0 + (uint64_t)q * 64 + lane;
        sum += j < c1 ? (osdo[s + j] >> HP_SDO_SH) & 0xffull : 0ull;
      }
    }
    sum = wave_sum(sum);
    if (lane == 0) s_sum[wv] = sum;
    __syncthreads();
    uint64_t carry = 0;
    for (int w = 0; w < wv; ++w) carry += s_sum[w];
    for (uint64_t j0 = c0; j0 < c1; j0 += 64 * U) {
      uint64_t xq[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const uint64_t j = j0 + (uint64_t)q * 64 + lane;
        xq[q] = j < c1 ? (osdo[s + j] >> HP_SDO_SH) & 0xffull : 0ull;
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const uint64_t j = j0 + (uint64_t)q * 64 + lane;
        const uint64_t in = wave_incl_scan(xq[q]) + carry;
        if (j < c1) pn[s + j] = (uint32_t)in;
        carry = __shfl(in, 63, 64);
      }
    }
    __syncthreads();
  }
}

// k_sl_rows: a thread per row of the range: |S(u)| = the length of the row's
// prefix of classes <= H (galloping, then binary search: a few dependent byte
// probes for most rows, ~2 log2 |list| for a hub), W+(u) = pn at its end.
// Writes W+(u) and |S(u)| directly (no atomics, no unpack).
__global__ void k_sl_rows(const uint64_t* __restrict__ lo, const uint8_t* __restrict__ cls,
                          const uint32_t* __restrict__ pn, uint32_t H, uint64_t ua, uint64_t nU,
                          uint32_t* __restrict__ cnt, unsigned long long* __restrict__ wu) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nU; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = lo[ua + r], e = lo[ua + r + 1];
    uint64_t a = s, b = e, step = 1;  // [s, a) <= H; the end of the prefix lies in [a, b]
    while (a < b) {
      const uint64_t p = a + step - 1 < b - 1 ? a + step - 1 : b - 1;
      if (cls[p] <= H) {
        a = p + 1;
        step <<= 1;
      } else {
        b = p;
        break;
      }
    }
    while (a < b) {
      const uint64_t m = (a + b) >> 1;
      if (cls[m] <= H) a = m + 1; else b = m;
    }
    cnt[r] = (uint32_t)(a - s);
    wu[r] = a > s ? pn[a - 1] : 0u;
  }
}

// The same W(u) from the survivors' side, for small H: the surviving
// intermediates are a prefix of the degree-class index (vbydeg, degrees 1..H),
// and every entry u of I(v) (the transposed multiset: one per occurrence of v
// in N(u)) adds deg v to W(u) -- P_H = sum of their degrees atomics instead of
// a pass over all M entries with a random degree gather each (C4 at H = 16:
// ~1e7 in-edges instead of 3.5e9 entries).  The same walk builds the
// survivor lists S(u) the row kernels then use instead of N(u).
// The survivor lists S(u) of a range: count per source (and W(u) with it),
// then, after a scan of the counts, fill (slots by a per-source cursor).
template <bool FILL>
__global__ __launch_bounds__(NT) void k_hp_surv_lists(GraphView g, const uint32_t* __restrict__ surv, uint64_t nsurv,
                                                      uint64_t ua, uint64_t ub, unsigned long long* __restrict__ wu,
                                                      uint32_t* __restrict__ cnt, const uint64_t* __restrict__ soff,
                                                      uint32_t* __restrict__ skeys) {
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < nsurv; i += (uint64_t)gridDim.x * NT) {
    const uint32_t v = surv[i];
    const unsigned long long d = g.deg[v];
    const uint64_t a = g.toff[v], b = g.toff[v + 1];
    for (uint64_t e0 = a; e0 < b; e0 += 8) {  // 8 in-edges in flight: keys, then the atomics, then the stores
      uint64_t u[8];
      bool in[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        u[q] = e0 + q < b ? g.tkeys[e0 + q] : 0ull;
        in[q] = e0 + q < b && u[q] >= ua && u[q] < ub;
      }
      if (FILL) {
        uint32_t p[8];
        uint64_t o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          p[q] = in[q] ? atomicAdd(&cnt[u[q] - ua], 1u) : 0u;
          o[q] = in[q] ? soff[u[q] - ua] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (in[q]) skeys[o[q] + p[q]] = v;
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (in[q]) {
            atomicAdd(&wu[u[q] - ua], d);
            atomicAdd(&cnt[u[q] - ua], 1u);
          }
      }
    }
  }
}

// The row's bin from W(u) and its degree (a wave walks N(u) in bin 0, so bin 0
// also bounds the degree); -1: no wedge.
__device__ __forceinline__ int hp_row_bin(uint64_t W, uint64_t du, int minbin, uint64_t b1max) {
  int b = W == 0 ? -1 : (W <= HP_B0_MAX && du <= HP_B0_DEG) ? 0 : W <= b1max ? 1 : W <= HP_B2_MAX ? 2 : 3;
  if (b >= 0 && b < minbin) b = minbin;  // test hook: route rows to a larger bin
  return b;
}

// The bins' row lists, ascending (the chunking searches them), as one stable
// partition of the range: tiles of HP_BTILE rows (row tile * HP_BTILE + i * NT
// + t, i < 8).  COUNT: per tile and bin its rows, into tcnt[b * ntiles +
// tile]; a scan gives tpos; SCATTER: every row at tpos[b * ntiles + tile] -
// tpos[b * ntiles] + its rank in the tile (substep, wave, lane order), and the
// bins' sizes into nl[b].  Round 3 wrote a flag byte per row and bin and
// scanned and scattered each bin (C4 H=16: 1.7 ms).
constexpr int HP_BIPT = 8;
constexpr uint64_t HP_BTILE = (uint64_t)NT * HP_BIPT;
template <bool SCATTER>
__global__ __launch_bounds__(NT) void k_hp_bins(const uint64_t* __restrict__ off, uint64_t ua, uint64_t nU,
                                                const uint64_t* __restrict__ wu, int minbin, uint64_t b1max,
                                                uint32_t* __restrict__ tcnt, const uint64_t* __restrict__ tpos,
                                                uint32_t* __restrict__ l0, uint32_t* __restrict__ l1,
                                                uint32_t* __restrict__ l2, uint32_t* __restrict__ l3,
                                                uint64_t* __restrict__ nl) {
  __shared__ uint32_t s_n[NWAVE][HP_NBINS];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t ntiles = (nU + HP_BTILE - 1) / HP_BTILE;
  if (SCATTER && blockIdx.x == 0 && t < HP_NBINS) nl[t] = tpos[(t + 1) * ntiles] - tpos[t * ntiles];
  uint32_t* L[HP_NBINS] = {l0, l1, l2, l3};
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int bn[HP_BIPT];
#pragma unroll
    for (int i = 0; i < HP_BIPT; ++i) {  // the tile's loads first: eight rows in flight per thread
      const uint64_t r = tile * HP_BTILE + (uint64_t)i * NT + t;
      bn[i] = r < nU ? hp_row_bin(wu[r], off[ua + r + 1] - off[ua + r], minbin, b1max) : -1;
    }
    uint32_t run[HP_NBINS] = {0, 0, 0, 0};  // the tile's rows per bin before this substep
    uint64_t base[HP_NBINS];
    if (SCATTER)
#pragma unroll
      for (int b = 0; b < HP_NBINS; ++b) base[b] = tpos[b * ntiles + tile] - tpos[b * ntiles];
#pragma unroll
    for (int i = 0; i < HP_BIPT; ++i) {
      uint64_t m[HP_NBINS];
#pragma unroll
      for (int b = 0; b < HP_NBINS; ++b) m[b] = __ballot(bn[i] == b);
      if (lane == 0)
#pragma unroll
        for (int b = 0; b < HP_NBINS; ++b) s_n[wv][b] = (uint32_t)__popcll(m[b]);
      __syncthreads();
      uint32_t tot[HP_NBINS], pre[HP_NBINS];
#pragma unroll
      for (int b = 0; b < HP_NBINS; ++b) {
        tot[b] = 0;
        pre[b] = 0;
        for (int w = 0; w < NWAVE; ++w) {
          const uint32_t c = s_n[w][b];
          pre[b] += w < wv ? c : 0u;
          tot[b] += c;
        }
      }
      if (SCATTER && bn[i] >= 0) {
        const int b = bn[i];
        const uint64_t r = tile * HP_BTILE + (uint64_t)i * NT + t;
        L[b][base[b] + run[b] + pre[b] + (uint32_t)__popcll(m[b] & ((1ull << lane) - 1ull))] = (uint32_t)(ua + r);
      }
#pragma unroll
      for (int b = 0; b < HP_NBINS; ++b) run[b] += tot[b];
      __syncthreads();
    }
    if (!SCATTER && t < HP_NBINS) tcnt[t * ntiles + tile] = run[t];
  }
}

// Chunk end: the largest r1 in (r0, nU] with wpre[r1] - wpre[r0] <= target
// (at least r0 + 1), and per bin the number of listed rows below ua + r1.
__global__ void k_hp_bounds(const uint64_t* __restrict__ wpre, uint64_t nU, uint64_t r0, uint64_t target, uint64_t ua,
                            const uint32_t* __restrict__ l0, const uint32_t* __restrict__ l1,
                            const uint32_t* __restrict__ l2, const uint32_t* __restrict__ l3,
                            const uint64_t* __restrict__ nl, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t base = wpre[r0];
  uint64_t lo = r0 + 1, hi = nU;  // answer in [lo, hi]
  while (lo < hi) {
    const uint64_t m = (lo + hi + 1) >> 1;
    if (wpre[m] - base <= target) lo = m; else hi = m - 1;
  }
  const uint64_t r1 = lo;
  out[0] = r1;
  const uint32_t* L[4] = {l0, l1, l2, l3};
  const uint64_t x = ua + r1;
  for (int b = 0; b < 4; ++b) {
    uint64_t a = 0, c = nl[b];
    while (a < c) {
      const uint64_t m = (a + c) >> 1;
      if ((uint64_t)L[b][m] < x) a = m + 1; else c = m;
    }
    out[1 + b] = a;
  }
}

// ---------------------------------------------------------------- bin 0: wave per row, LDS table
// Bin 0 is split into table-size tiers (HP_TIER_W): a row of W(u) <= 128 needs
// at most a 256-entry table, and the LDS of a 1024-entry table per wave
// (45 KB per workgroup) holds the kernel to 3 waves per SIMD -- too few to
// hide the random graph reads of a small row.  k_hp_tier partitions the
// chunk's bin-0 rows by tier (order within a tier is free: candidates are
// emitted unordered), and one k_hp_wave<TW> launch per tier reads its slice
// and row count from the device.
constexpr int HP_NTIER = 3;
__host__ __device__ constexpr uint64_t hp_tier_w(int t) { return t == 0 ? 128 : t == 1 ? 256 : HP_B0_MAX; }

// tcnt: [0, 3) rows per tier (counted by the first pass), [3, 6) cursors.
// A workgroup counts its rows per tier and (SCATTER) reserves its slots with
// one global atomic per tier, then places its rows from LDS running offsets
// (round 3 reserved per 256 rows: 6e5 atomics on three words serialised at
// their L2 channel, 0.9 ms of the C4 H=16 call).
template <bool SCATTER>
__global__ __launch_bounds__(NT) void k_hp_tier(const uint32_t* __restrict__ rows, uint64_t nrows,
                                                const uint64_t* __restrict__ wu, uint64_t ua,
                                                uint32_t* __restrict__ tcnt, uint32_t* __restrict__ out,
                                                uint64_t w0 = hp_tier_w(0), uint64_t w1 = hp_tier_w(1)) {
  __shared__ uint32_t s_n[NWAVE][HP_NTIER];
  __shared__ uint32_t s_base[HP_NTIER];
  const int lane = lane_id(), wv = wave_id();
  auto tier_of = [&](uint64_t i, uint32_t* pu) -> int {
    if (i >= nrows) return -1;
    const uint32_t u = rows[i];
    *pu = u;
    const uint64_t W = wu[u - ua];
    return W <= w0 ? 0 : W <= w1 ? 1 : 2;
  };
  uint32_t cnt[HP_NTIER] = {0, 0, 0};  // this wave's rows per tier (lane 0)
  for (uint64_t b0 = (uint64_t)blockIdx.x * NT; b0 < nrows; b0 += (uint64_t)gridDim.x * NT) {
    uint32_t u = 0;
    const int t = tier_of(b0 + threadIdx.x, &u);
#pragma unroll
    for (int q = 0; q < HP_NTIER; ++q) {
      const uint64_t m = __ballot(t == q);  // every lane votes (a ballot under `lane == 0 ?` would see one lane)
      cnt[q] += lane == 0 ? (uint32_t)__popcll(m) : 0u;
    }
  }
  if (lane == 0)
    for (int q = 0; q < HP_NTIER; ++q) s_n[wv][q] = cnt[q];
  __syncthreads();
  if (threadIdx.x < HP_NTIER) {
    uint32_t tot = 0;
    for (int w = 0; w < NWAVE; ++w) tot += s_n[w][threadIdx.x];
    if (!SCATTER && tot) atomicAdd(&tcnt[threadIdx.x], tot);
    if (SCATTER) {
      uint32_t tb = 0;
      for (int q = 0; q < (int)threadIdx.x; ++q) tb += tcnt[q];
      s_base[threadIdx.x] = tb + (tot ? atomicAdd(&tcnt[HP_NTIER + threadIdx.x], tot) : 0u);
    }
  }
  if (!SCATTER) return;
  __syncthreads();
  for (uint64_t b0 = (uint64_t)blockIdx.x * NT; b0 < nrows; b0 += (uint64_t)gridDim.x * NT) {
    uint32_t u = 0;
    const int t = tier_of(b0 + threadIdx.x, &u);
    uint64_t m[HP_NTIER];
#pragma unroll
    for (int q = 0; q < HP_NTIER; ++q) m[q] = __ballot(t == q);
    if (lane == 0)
      for (int q = 0; q < HP_NTIER; ++q) s_n[wv][q] = (uint32_t)__popcll(m[q]);
    __syncthreads();
    if (t >= 0) {
      uint32_t pre = 0;
      for (int w = 0; w < wv; ++w) pre += s_n[w][t];
      out[s_base[t] + pre + (uint32_t)__popcll(m[t] & ((1ull << lane) - 1))] = u;
    }
    __syncthreads();
    if (threadIdx.x < HP_NTIER) {
      uint32_t tot = 0;
      for (int w = 0; w < NWAVE; ++w) tot += s_n[w][threadIdx.x];
      s_base[threadIdx.x] += tot;
    }
    __syncthreads();
  }
}

template <bool CUSTOM, int TW = HP_WT, int STG = HP_STG, bool KD = false>
__global__ __launch_bounds__(NT) void k_hp_wave(HpArgs a, const uint32_t* __restrict__ rows, uint64_t nrows,
                                                const uint64_t* __restrict__ wu, uint64_t ua,
                                                const uint32_t* __restrict__ tcnt = nullptr, int tier = 0) {
  constexpr int VT = CUSTOM ? TW : 1;
  __shared__ uint32_t s_k[NWAVE][TW];
  __shared__ uint32_t s_c[NWAVE][TW];
  __shared__ uint32_t s_v0[NWAVE][VT];
  __shared__ uint32_t s_v1[NWAVE][VT];
  __shared__ uint32_t s_incl[NWAVE][64];
  __shared__ uint64_t s_start[NWAVE][64];
  __shared__ uint32_t s_iv[NWAVE][64];
  __shared__ uint32_t s_gu[NWAVE][STG], s_gw[NWAVE][STG];
  __shared__ float s_gs[NWAVE][STG];
  constexpr int SK = CUSTOM ? TW / 2 : 1;  // AA / RA: S(u) sorted (|S(u)| <= W(u) <= TW / 2)
  __shared__ uint32_t s_sk[NWAVE][SK];
  __shared__ double s_ic[NWAVE][CUSTOM ? 64 : 1];
  const int lane = lane_id(), wv = wave_id();
  if (tcnt) {  // tier slice of the partitioned list
    uint32_t base = 0;
    for (int r = 0; r < tier; ++r) base += tcnt[r];
    rows += base;
    nrows = tcnt[tier];
  }
  const HpTable tb{s_k[wv], s_c[wv], s_v0[wv], s_v1[wv]};
  for (int i = lane; i < TW; i += 64) {
    s_k[wv][i] = HP_EMPTY;
    s_c[wv][i] = 0;
    if (CUSTOM) s_v0[wv][i] = 0;  // owner tokens (ordered accumulation)
  }
  HpStage sg{s_gu[wv], s_gw[wv], s_gs[wv], STG, 0, 0, 0};
  const int64_t tau = *a.tau;
  uint64_t wedges = 0;
  wave_sync_lds();
  for (uint64_t ri = (uint64_t)blockIdx.x * NWAVE + wv; ri < nrows; ri += (uint64_t)gridDim.x * NWAVE) {
    const uint32_t u = rows[ri];
    const uint64_t W = wu[u - ua];
    const int lg = max(6, log2_ceil(2 * W));
    const uint32_t T = 1u << lg, mask = T - 1;
    if (T > (uint32_t)TW) {  // a row outside this tier (a partition bug): fail the call, never overrun LDS
      if (lane == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
      continue;
    }
    const int shift = 32 - lg;
    const uint64_t o0 = a.g.off[u], o1 = a.g.off[u + 1];
    const uint64_t du = o1 - o0;
    const uint32_t* fh;
    uint64_t nf;
    hp_first_hops(a, u, o0, du, &fh, &nf);
    if (CUSTOM && a.soff && !a.ssorted) {  // S(u) from in-edge atomics is unordered: sort it
      if (nf > (uint64_t)SK) {
        if (lane == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
        continue;
      }
      const uint32_t n2 = pow2_at_least((uint32_t)nf);
      for (uint32_t e = (uint32_t)lane; e < n2; e += 64) s_sk[wv][e] = e < nf ? fh[e] : 0xffffffffu;
      wave_sync_lds();
      wave_bitonic_u32(s_sk[wv], n2);
      fh = s_sk[wv];
    }
    uint32_t round = 0;
    // packed survivor entries (the part of N(v) above u, no row-bound gather)
    const uint64_t* fd = a.sdo && fh != s_sk[wv] && a.soff ? a.sdo + (fh - a.skeys) : nullptr;
    for (uint64_t base = 0; base < nf; base += 64) {
      const uint64_t i = base + lane;
      uint32_t len = 0, v = 0;
      uint64_t st = 0;
      double cv = 0.0;
      if (i < nf) {
        if (fd) {
          const uint64_t x = fd[i];
          len = (uint32_t)(x >> HP_SDO_SH) & 0xffu;
          st = x & ((1ull << HP_SDO_SH) - 1);
          if (CUSTOM) cv = a.g.ctab[x >> 48];
        } else {
          v = fh[i];
          const uint32_t d = a.g.deg[v];
          if (hp_surv(d, a.H)) {
            len = d;
            st = a.g.off[v];
            if (CUSTOM) cv = a.g.ctab[d];
          }
        }
      }
      const uint32_t incl = (uint32_t)wave_incl_scan(len);
      s_incl[wv][lane] = incl;
      s_start[wv][lane] = st;
      s_iv[wv][lane] = v;
      if (CUSTOM) s_ic[wv][lane] = cv;
      wave_sync_lds();
      const uint32_t total = __shfl(incl, 63, 64);
      if constexpr (CUSTOM) {
        hp_wedges<64, true>(total, (uint32_t)lane, 64u, s_incl[wv], s_start[wv], s_iv[wv], a.g.keys,
                            [&](bool ok, uint32_t w, uint32_t ent) {
                              const bool in = ok && w > u;
                              uint32_t h = 0;
                              if (in) {
                                ++wedges;
                                h = ho_find(tb, mask, shift, w, &a.ctr[HPC_ERR]);
                              }
                              ho_add_wave(tb, in, h, s_ic[wv][ent], &round);
                            });
      } else if constexpr (KD) {  // TW <= 1024: at most 512 wedges per row, counts in 10 bits
        hp_wedges<64, false, true>(total, (uint32_t)lane, 64u, s_incl[wv], s_start[wv], s_iv[wv], a.g.keys,
                                   [&](uint32_t w, uint32_t, uint32_t dw) {
                                     if (w > u) {
                                       ++wedges;
                                       hp_insert_kd<10>(tb, mask, shift, w, dw, &a.ctr[HPC_ERR]);
                                     }
                                   }, a.kdeg);
      } else {
        hp_wedges<64>(total, (uint32_t)lane, 64u, s_incl[wv], s_start[wv], s_iv[wv], a.g.keys,
                      [&](uint32_t w, uint32_t v) {
                        if (w > u) {
                          ++wedges;
                          hp_insert<false, CUSTOM>(tb, mask, shift, w, v, &a.ctr[HPC_ERR]);
                        }
                      });
      }
      wave_sync_lds();
    }
    // first-order exclusion (predict.hxx:306-307): the entries of N(u) above u
    // marked, or tested in the membership table at the drain (a slice beyond
    // HB_XF times the row's wedge bound)
    const uint32_t xu = a.xs ? a.xs[u] : 0u;
    const bool ux = hp_use_etab(a, du - xu, W);
    if (!ux)
      hp_stream(a.g.keys + o0 + xu, du - xu, (uint32_t)lane, 64u, [&](uint32_t x) {
        if (x > u) hp_mark<false>(tb, mask, shift, x);
      });
    wave_sync_lds();
    hp_drain<false, CUSTOM, 8, CUSTOM, KD ? 10 : 0>(tb, T, (uint32_t)lane, 64u, sg, a, u, du, tau, ux);
    wave_sync_lds();
  }
  hp_finish(sg, a, wedges);
}

// ---------------------------------------------------------------- bin 0: row batches
// A wave per row leaves most of a small row's lanes idle and pays the row's
// chain of dependent graph reads (row bounds -> S(u) -> deg/off of v -> N(v)
// -> deg w -> emission) once per row.  With the survivor lists S(u) (small H)
// the rows of a tier are instead taken in batches: consecutive rows of the
// list while sum (W(u) + HB_ROWCOST) stays within TW / 4 (tiers 0 and 1:
// W(u) <= TW / 4 each), so a batch has
// at most TW / 20 < 64 rows and at most TW / 2 wedges.  One wave accumulates a
// whole batch in one LDS table keyed (slot << wbits | w), slot = the row's
// index in the batch, and pays the chain once per batch.  Exclusion marks
// (slot, x) for x in N(u); the drain decodes the slot back to (u, deg u).
// Needs S <= 2^(32 - 6) (six slot bits above w).
constexpr uint64_t HB_ROWCOST = 5;  // budget units per row besides its wedges (bounds the rows per batch)

constexpr int HB_UN = 8;            // loads per lane in flight in the batch loops (a batch is a few round trips)
constexpr int HB_EP = 4;            // membership-table probes in flight per lane in the batch drain

// The rows of tiers tlo..thi: a contiguous region of the tier list.
__device__ __forceinline__ void hb_region(const uint32_t* tcnt, int tlo, int thi, uint32_t* base, uint32_t* cnt) {
  uint32_t b = 0, c = 0;
  for (int r = 0; r < tlo; ++r) b += tcnt[r];
  for (int r = tlo; r <= thi; ++r) c += tcnt[r];
  *base = b;
  *cnt = c;
}

// bw[i] = W(u_i) + HB_ROWCOST for the rows of tiers tlo..thi of the tier list, 0 beyond
__global__ void k_hp_batch_w(const uint32_t* __restrict__ tl, uint64_t n0, const uint32_t* __restrict__ tcnt,
                             int tlo, int thi, const uint64_t* __restrict__ wu, uint64_t ua, uint64_t* __restrict__ bw) {
  uint32_t base, cnt;
  hb_region(tcnt, tlo, thi, &base, &cnt);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n0; i += (uint64_t)gridDim.x * blockDim.x)
    bw[i] = i < cnt ? wu[tl[base + i] - ua] + HB_ROWCOST : 0ull;
}

// bstart[b] = the first row whose budget prefix reaches b * BW (batch b = rows
// [bstart[b], bstart[b + 1])); *nbatch = the number of batches (zeroed first).
__global__ void k_hp_batch_starts(const uint64_t* __restrict__ bpre, const uint32_t* __restrict__ tcnt, int tlo,
                                  int thi, uint64_t bwid, uint32_t* __restrict__ bstart, uint32_t* __restrict__ nbatch) {
  uint32_t base, cnt;
  hb_region(tcnt, tlo, thi, &base, &cnt);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = bpre[i] / bwid;
    const uint64_t b0 = i ? bpre[i - 1] / bwid + 1 : 0;  // batches without a row start of their own begin here
    for (uint64_t q = b0; q <= b; ++q) bstart[q] = (uint32_t)i;
    if (i + 1 == cnt) {
      bstart[b + 1] = (uint32_t)cnt;
      *nbatch = (uint32_t)(b + 1);
    }
  }
}

// hp_wedges with the first-hop entry's index: f(w, v, entry), UN keys per lane in flight
// (ALL: f(ok, w, v, entry) on every lane, wave-convergent, for the ordered accumulation)
// (KD: also the degree of every second hop, kd[] = the graph's entry degrees,
// loaded beside the key: f(w, v, entry, deg w))
template <int UN, bool ALL = false, bool KD = false, typename IT, typename F>
__device__ __forceinline__ void hb_wedges(uint64_t total, uint32_t t, const IT* s_incl, const uint64_t* s_start,
                                          const uint32_t* s_iv, const uint32_t* keys, F f,
                                          const uint32_t* kd = nullptr) {
  // the steps past the batch's wedges are skipped wave-uniformly (a batch often
  // holds fewer than 64 * UN wedges: their searches and loads would be issued anyway)
  const uint32_t tot = __builtin_amdgcn_readfirstlane((uint32_t)total);
  for (uint64_t j0 = 0; j0 < tot; j0 += (uint64_t)64 * UN) {
    uint32_t w[UN], v[UN], e[UN], dw[UN];
    bool ok[UN];
    const uint32_t nq = (uint32_t)min((uint64_t)UN, (tot - j0 + 63) / 64);
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      if ((uint32_t)q >= nq) break;
      const uint64_t j = j0 + (uint64_t)q * 64 + t;
      ok[q] = j < total;
      uint32_t lo = 0;  // the first entry with s_incl > j (six fixed steps, see hb_slot)
#pragma unroll
      for (uint32_t bit = 32; bit > 0; bit >>= 1) lo += (uint64_t)s_incl[lo + bit - 1] <= j ? bit : 0u;
      if (lo > 63) lo = 63;
      const uint64_t ex = lo ? (uint64_t)s_incl[lo - 1] : 0ull;
      v[q] = s_iv[lo];
      e[q] = lo;
      const uint64_t at = ok[q] ? s_start[lo] + (j - ex) : 0ull;
      w[q] = keys[at];
      if constexpr (KD) dw[q] = kd[at];
    }
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      if ((uint32_t)q >= nq) break;
      if constexpr (ALL) f(ok[q], w[q], v[q], e[q]);
      else if constexpr (KD) { if (ok[q]) f(w[q], v[q], e[q], dw[q]); }
      else if (ok[q]) f(w[q], v[q], e[q]);
    }
  }
}


// the batch slot of flattened item j < incl[63]: the first r with incl[r] > j
// (64 non-decreasing inclusive prefixes; lanes past the batch's rows repeat
// the total).  Six fixed steps, no loop: the search runs for every item and a
// data-dependent loop costs more in branch and exec-mask instructions than the
// compares themselves.
__device__ __forceinline__ uint32_t hb_slot(const uint32_t* incl, uint32_t, uint32_t j) {
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t bit = 32; bit > 0; bit >>= 1) lo += incl[lo + bit - 1] <= j ? bit : 0u;
  return lo;
}

// ---------------------------------------------------------------- one-word table entries (count metrics)
// The row batches' count tables keep an entry as ONE u64 word, key << 32 |
// count word, so a wedge that creates its entry costs a single LDS
// compare-and-swap (the two-array table paid a key load, a key CAS and a
// count add): most wedges of a k-filling call create their entry (C4 JAC
// H=16: 2.77e8 candidates from 2.80e8 wedges).  The count word is the KD
// layout (count in the low CB bits, min(deg w, DSAT) above, HP_EXCL on top),
// so an add of 1 never carries into the key.
constexpr uint64_t HP_EMPTY64 = (uint64_t)HP_EMPTY << 32;

template <int CB>
__device__ __forceinline__ void h64_insert(uint64_t* t, uint32_t mask, int shift, uint32_t key, uint32_t dw,
                                           unsigned long long* err) {
  constexpr uint32_t DSAT = CB > 0 ? (1u << (31 - CB)) - 1u : 0u;
  const uint64_t init = (uint64_t)key << 32 | (1u + (CB > 0 ? (dw < DSAT ? dw : DSAT) << CB : 0u));
  uint32_t h = hp_hash(key, shift);
  for (uint32_t probe = 0;; ++probe) {
    if (probe > mask) { atomicOr(err, 1ull); return; }
    const uint64_t old = atomicCAS((unsigned long long*)&t[h], (unsigned long long)HP_EMPTY64, (unsigned long long)init);
    if (old == HP_EMPTY64) return;
    if ((uint32_t)(old >> 32) == key) {
      atomicAdd((unsigned long long*)&t[h], 1ull);
      return;
    }
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ void h64_mark(uint64_t* t, uint32_t mask, int shift, uint32_t x) {
  uint32_t h = hp_hash(x, shift);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const uint64_t cur = *(volatile uint64_t*)&t[h];
    const uint32_t k = (uint32_t)(cur >> 32);
    if (k == x) { atomicOr((unsigned long long*)&t[h], (unsigned long long)HP_EXCL); return; }
    if (k == HP_EMPTY) return;
    h = (h + 1) & mask;
  }
}

// KD (count metrics, with the graph's entry degrees): deg w rides in the table
// (hp_insert_kd<10>: a batch holds at most 512 wedges), no gather at the drain.
template <bool CUSTOM, int TW, int STG = HP_STG, bool KD = false, int UN = HB_UN, int MW = 1>
__global__ __launch_bounds__(NT, MW) void k_hp_batch(HpArgs a, const uint32_t* __restrict__ tl,
                                                 const uint32_t* __restrict__ tcnt, int tlo, int thi,
                                                 const uint32_t* __restrict__ bstart,
                                                 const uint32_t* __restrict__ nbatch, const uint64_t* __restrict__ wu,
                                                 uint64_t ua, int wbits) {
  constexpr int VT = CUSTOM ? TW : 1;
  constexpr int KT = CUSTOM ? TW : 1;      // AA / RA: key and accumulator arrays (ordered tables)
  __shared__ uint32_t s_k[NWAVE][KT];
  __shared__ uint32_t s_c[NWAVE][KT];
  __shared__ uint64_t s_kc[NWAVE][CUSTOM ? 1 : TW];  // count metrics: one-word entries
  __shared__ uint32_t s_v0[NWAVE][VT];
  __shared__ uint32_t s_v1[NWAVE][VT];
  __shared__ uint32_t s_incl[NWAVE][64];   // first-hop block: inclusive prefix of the lengths
  __shared__ uint64_t s_start[NWAVE][64];
  __shared__ uint32_t s_iv[NWAVE][64];
  __shared__ uint32_t s_islot[NWAVE][64];
  __shared__ uint32_t s_u[NWAVE][64];      // batch rows: u, deg u, S(u) / N(u) starts, inclusive prefixes
  __shared__ uint32_t s_du[NWAVE][64];
  __shared__ uint64_t s_s0[NWAVE][64];
  __shared__ uint64_t s_o0[NWAVE][64];
  __shared__ uint32_t s_sp[NWAVE][64];
  __shared__ uint32_t s_np[NWAVE][64];
  __shared__ uint8_t s_ux[NWAVE][64];     // the row's entries tested in the membership table
  __shared__ uint32_t s_gu[NWAVE][STG], s_gw[NWAVE][STG];
  __shared__ float s_gs[NWAVE][STG];
  constexpr int SK = CUSTOM ? TW / 2 : 1;  // AA / RA: the batch's first hops (slot << wbits | v), sorted
  __shared__ uint32_t s_sk[NWAVE][SK];
  __shared__ double s_ic[NWAVE][CUSTOM ? 64 : 1];
  const int lane = lane_id(), wv = wave_id();
  uint32_t base, cnt;
  hb_region(tcnt, tlo, thi, &base, &cnt);
  const uint32_t* rows = tl + base;
  const uint32_t nb = *nbatch;
  const uint32_t wmask = (1u << wbits) - 1u;
  const HpTable tb{s_k[wv], s_c[wv], s_v0[wv], s_v1[wv]};
  uint64_t* const t64 = s_kc[wv];
  for (int i = lane; i < TW; i += 64) {
    if (CUSTOM) {
      s_k[wv][i] = HP_EMPTY;
      s_c[wv][i] = 0;
      s_v0[wv][i] = 0;  // owner tokens
    } else {
      t64[i] = HP_EMPTY64;
    }
  }
  uint32_t round = 0;
  HpStage sg{s_gu[wv], s_gw[wv], s_gs[wv], STG, 0, 0, 0, 0, 0, 0, a.win != 0, 0};
  const int64_t tau = *a.tau;
  uint64_t wedges = 0;
  uint64_t abytes = 0;  // algorithmic bytes (wave-uniform): rows, entries, exclusion keys
  uint64_t drained = 0;  // per lane: table entries whose deg w is gathered (count metrics without KD)
  uint64_t etq = 0;      // per lane: membership-table tests (8 bytes each: the key)
  wave_sync_lds();
  // The next batch's bounds, rows and row data are loaded while this batch
  // works (bounds during the first hops, rows during the exclusion, row data
  // before the drain), so a batch pays only its own chain of graph reads.
  const uint32_t stride = gridDim.x * NWAVE;
  uint32_t b = blockIdx.x * NWAVE + wv;
  uint32_t r0 = 0, nr = 0, u = 0, ns = 0, du = 0;
  uint64_t s0 = 0, o0 = 0, W = 0;
  auto fetch_bounds = [&](uint32_t bb, uint32_t* q0, uint32_t* qn) {
    *q0 = bb < nb ? bstart[bb] : 0u;
    *qn = bb < nb ? bstart[bb + 1] - *q0 : 0u;  // < 64 by the budget
  };
  // per row: W+(u), S(u) bounds, deg u (the score) and the exclusion slice of
  // N(u) -- its entries above u, [o0, o0 + dx)
  auto fetch_info = [&](uint32_t n, uint32_t uu, uint64_t* pW, uint64_t* ps0, uint32_t* pns, uint64_t* po0,
                        uint32_t* pdu, uint32_t* pdx) {
    if ((uint32_t)lane < n) {
      *pW = wu[uu - ua];
      *ps0 = a.soff[uu - a.sua];
      *pns = (uint32_t)hp_slen(a, uu, *ps0);
      const uint64_t ob = a.g.off[uu];
      *pdu = (uint32_t)(a.g.off[uu + 1] - ob);
      const uint32_t xu = a.xs ? a.xs[uu] : 0u;
      *po0 = ob + xu;
      *pdx = *pdu - xu;
    } else {
      *pW = 0;
      *ps0 = 0;
      *pns = 0;
      *po0 = 0;
      *pdu = 0;
      *pdx = 0;
    }
  };
  uint32_t dx = 0;
  fetch_bounds(b, &r0, &nr);
  u = (uint32_t)lane < nr ? rows[r0 + lane] : 0u;
  fetch_info(nr, u, &W, &s0, &ns, &o0, &du, &dx);
  uint64_t ph_t = a.ph ? __builtin_amdgcn_s_memrealtime() : 0, ph_acc[4] = {0, 0, 0, 0};
  auto ph_mark = [&](int i) {  // time since the last mark goes to phase i
    if (a.ph) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      ph_acc[i] += now - ph_t;
      ph_t = now;
    }
  };
  for (; b < nb;) {
    const uint32_t bn = b + stride;
    uint32_t pr0, pnr, pu = 0;
    if (nr == 0) {  // an empty batch (a row wider than the budget window skipped it)
      fetch_bounds(bn, &r0, &nr);
      u = (uint32_t)lane < nr ? rows[r0 + lane] : 0u;
      fetch_info(nr, u, &W, &s0, &ns, &o0, &du, &dx);
      b = bn;
      continue;
    }
    fetch_bounds(bn, &pr0, &pnr);
    const bool ux = hp_use_etab(a, dx, W);
    const uint32_t sp = (uint32_t)wave_incl_scan(ns), np = (uint32_t)wave_incl_scan(ux ? 0u : dx);
    s_ux[wv][lane] = ux ? 1 : 0;
    s_u[wv][lane] = u;
    s_du[wv][lane] = du;
    s_s0[wv][lane] = s0;
    s_o0[wv][lane] = o0;
    s_sp[wv][lane] = sp;
    s_np[wv][lane] = np;
    wave_sync_lds();
    const uint32_t NS = __shfl(sp, (int)nr - 1, 64), NN = __shfl(np, (int)nr - 1, 64);
    // per batch: its bounds (8); per row: list entry, W+(u), S(u) and N(u) bounds (28); per
    // survivor entry 8 (packed) or 12 (key, deg, off); per exclusion key 4
    abytes += 8 + 28ull * nr + (a.sdo ? 8ull : 12ull) * NS + 4ull * NN;
    const uint64_t Wb = wave_sum(W);
    const int lg = max(6, log2_ceil(2 * Wb));
    const uint32_t T = 1u << lg, mask = T - 1;
    if (T > (uint32_t)TW) {  // a batch beyond the budget (a partition bug): fail the call, never overrun LDS
      if (lane == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
      nr = 0;  // skip it; the next batch is fetched at the loop top
      continue;
    }
    const int shift = 32 - lg;
    if (CUSTOM && !a.sdo) {
      // AA / RA: the batch's first hops sorted by (slot, v) -- S(u) is unordered
      // -- so that the wedge steps run in the reference's order of additions
      if (NS > (uint32_t)SK) {  // more first hops than wedges (a budget bug): fail the call
        if (lane == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
        nr = 0;
        continue;
      }
      const uint32_t n2 = pow2_at_least(NS);
      for (uint32_t e = (uint32_t)lane; e < n2; e += 64) {
        uint32_t key = 0xffffffffu;
        if (e < NS) {
          const uint32_t slot = hb_slot(s_sp[wv], nr, e);
          const uint32_t ex = slot ? s_sp[wv][slot - 1] : 0u;
          key = (slot << wbits) | a.skeys[s_s0[wv][slot] + (e - ex)];
        }
        s_sk[wv][e] = key;
      }
      wave_sync_lds();
      if (!a.ssorted) wave_bitonic_u32(s_sk[wv], n2);
    }
    ph_mark(0);  // batch setup (row data wait, scans, AA order)
    // the batch's surviving first hops, 64 at a time; their wedges (slot, w) into the table
    for (uint32_t e0 = 0; e0 < NS; e0 += 64) {
      const uint32_t e = e0 + (uint32_t)lane;
      uint32_t len = 0, v = 0, slot = 0;
      uint64_t st = 0;
      double cv = 0.0;
      if (e < NS) {
        if (a.sdo) {  // packed survivor entries: no degree / offset gather (every entry survives)
          slot = hb_slot(s_sp[wv], nr, e);
          const uint32_t ex = slot ? s_sp[wv][slot - 1] : 0u;
          const uint64_t x = a.sdo[s_s0[wv][slot] + (e - ex)];
          len = (uint32_t)(x >> HP_SDO_SH) & 0xffu;  // the part of N(v) above u
          st = x & ((1ull << HP_SDO_SH) - 1);
          if (CUSTOM) cv = a.g.ctab[x >> 48];
        } else {
          if (CUSTOM) {
            const uint32_t key = s_sk[wv][e];
            slot = key >> wbits;
            v = key & wmask;
          } else {
            slot = hb_slot(s_sp[wv], nr, e);
            const uint32_t ex = slot ? s_sp[wv][slot - 1] : 0u;
            v = a.skeys[s_s0[wv][slot] + (e - ex)];
          }
          const uint32_t d = a.g.deg[v];
          if (hp_surv(d, a.H)) {
            len = d;
            st = a.g.off[v];
            if (CUSTOM) cv = a.g.ctab[d];
          }
        }
      }
      const uint32_t incl = (uint32_t)wave_incl_scan(len);
      s_incl[wv][lane] = incl;
      s_start[wv][lane] = st;
      s_iv[wv][lane] = v;
      s_islot[wv][lane] = slot;
      if (CUSTOM) s_ic[wv][lane] = cv;
      wave_sync_lds();
      const uint32_t total = __shfl(incl, 63, 64);
      if constexpr (CUSTOM) {
        hb_wedges<UN, true>(total, (uint32_t)lane, s_incl[wv], s_start[wv], s_iv[wv], a.g.keys,
                               [&](bool ok, uint32_t w, uint32_t, uint32_t ent) {
                                 const uint32_t sl = s_islot[wv][ent];
                                 const bool in = ok && w > s_u[wv][sl];
                                 uint32_t h = 0;
                                 if (in) {
                                   ++wedges;
                                   h = ho_find(tb, mask, shift, (sl << wbits) | w, &a.ctr[HPC_ERR]);
                                 }
                                 ho_add_wave(tb, in, h, s_ic[wv][ent], &round);
                               });
      } else if constexpr (KD) {
        hb_wedges<UN, false, true>(total, (uint32_t)lane, s_incl[wv], s_start[wv], s_iv[wv], a.g.keys,
                                      [&](uint32_t w, uint32_t, uint32_t ent, uint32_t dw) {
                                        const uint32_t sl = s_islot[wv][ent];
                                        if (w > s_u[wv][sl]) {
                                          ++wedges;
                                          h64_insert<10>(t64, mask, shift, (sl << wbits) | w, dw, &a.ctr[HPC_ERR]);
                                        }
                                      }, a.kdeg);
      } else {
        hb_wedges<UN>(total, (uint32_t)lane, s_incl[wv], s_start[wv], s_iv[wv], a.g.keys,
                         [&](uint32_t w, uint32_t vv, uint32_t ent) {
                           const uint32_t sl = s_islot[wv][ent];
                           if (w > s_u[wv][sl]) {
                             ++wedges;
                             h64_insert<0>(t64, mask, shift, (sl << wbits) | w, 0u, &a.ctr[HPC_ERR]);
                           }
                         });
      }
      wave_sync_lds();
    }
    ph_mark(1);  // first hops and wedge inserts
    pu = (uint32_t)lane < pnr ? rows[pr0 + lane] : 0u;  // the next batch's rows, in flight during the exclusion
    // first-order exclusion (predict.hxx:306-307): (slot, x) for x in N(u), x > u
    // (marking from N(u) measured faster here than a membership-table line per entry)
    // (prefetching the first block of these keys during the wedge phase measured
    // slower: 46.6 -> 52.7 ms on C3 JAC H=16)
    const uint32_t NNs = __builtin_amdgcn_readfirstlane(NN);
    for (uint32_t x0 = 0; x0 < NNs; x0 += 64 * UN) {
      uint32_t key[UN], sl[UN];
      const uint32_t nq = min((uint32_t)UN, (NNs - x0 + 63) / 64);
#pragma unroll
      for (int q = 0; q < UN; ++q) {
        if ((uint32_t)q >= nq) break;
        const uint32_t x = x0 + (uint32_t)q * 64 + (uint32_t)lane;
        sl[q] = x < NN ? hb_slot(s_np[wv], nr, x) : 0u;
        const uint32_t ex = sl[q] ? s_np[wv][sl[q] - 1] : 0u;
        key[q] = x < NN ? a.g.keys[s_o0[wv][sl[q]] + (x - ex)] : 0u;
      }
#pragma unroll
      for (int q = 0; q < UN; ++q) {
        if ((uint32_t)q >= nq) break;
        const uint32_t x = x0 + (uint32_t)q * 64 + (uint32_t)lane;
        if (x < NN && key[q] > s_u[wv][sl[q]]) {
          if (CUSTOM) hp_mark<false>(tb, mask, shift, (sl[q] << wbits) | key[q]);
          else h64_mark(t64, mask, shift, (sl[q] << wbits) | key[q]);
        }
      }
    }
    wave_sync_lds();
    ph_mark(2);  // exclusion
    uint64_t pW, ps0, po0;
    uint32_t pns, pdu, pdx;
    fetch_info(pnr, pu, &pW, &ps0, &pns, &po0, &pdu, &pdx);  // the next batch's row data, in flight during the drain
    // drain: every entry scored for its own row (a list of the claimed slots
    // instead of this scan measured slower: the claims cost more in the insert
    // loop than the scan of empty slots)
    const uint32_t Ts = __builtin_amdgcn_readfirstlane(T);
    for (uint32_t i0 = 0; i0 < Ts; i0 += 64 * UN) {
      uint32_t kq[UN], c[UN], v0[UN], v1[UN], dw[UN];
      const uint32_t nq = min((uint32_t)UN, (Ts - i0) / 64);  // T: a power of two >= 64
#pragma unroll
      for (int q = 0; q < UN; ++q) {
        if ((uint32_t)q >= nq) break;
        const uint32_t i = i0 + (uint32_t)q * 64 + (uint32_t)lane;
        c[q] = v0[q] = v1[q] = 0;
        if (CUSTOM) {
          kq[q] = ho_take(tb, i, &c[q]);
        } else {
          const uint64_t x = t64[i];
          kq[q] = (uint32_t)(x >> 32);
          c[q] = (uint32_t)x;
          if (kq[q] != HP_EMPTY) t64[i] = HP_EMPTY64;
        }
      }
      if (!CUSTOM) {
#pragma unroll
        for (int q = 0; q < UN; ++q) {
          if ((uint32_t)q >= nq) break;
          const uint32_t w = kq[q] != HP_EMPTY ? (kq[q] & wmask) : 0u;
          dw[q] = KD ? hp_kd_deg<10>(a.g, c[q], w) : a.g.deg[w];
        }
      }
      // first-order exclusion by the membership table for the entries of
      // table-tested rows (count tables: two first buckets in flight at a time;
      // the tests deferred to a separate high-occupancy kernel after the chunk
      // measured slower: C4 JAC H=16 43.4 -> 48.1 ms, the kernel 13.9 -> 9.7 ms
      // but the deferred probes ~9 ms -- a random 64-byte line per test, no
      // longer hidden behind the batches' own latency)
      // (count tables: HB_EP first buckets in flight at a time)
      constexpr int EP = CUSTOM ? 2 : HB_EP;
#pragma unroll
      for (int q0 = 0; q0 < UN; q0 += EP) {
        if ((uint32_t)q0 >= nq) break;
        uint64_t ek[EP];
        bool ea[EP], er[EP];
#pragma unroll
        for (int z = 0; z < EP; ++z) {
          const int q = q0 + z;
          const bool valid = q < UN && (uint32_t)q < nq && kq[q] != HP_EMPTY;
          const uint32_t sl = valid ? kq[q] >> wbits : 0u;
          ea[z] = valid && s_ux[wv][sl];
          ek[z] = ea[z] ? ((uint64_t)s_u[wv][sl] << 32 | (kq[q] & wmask)) : 0ull;
        }
        if (CUSTOM) {
#pragma unroll
          for (int z = 0; z < EP; ++z) er[z] = ea[z] && et_has(a.g.etab, a.g.etbits, (uint32_t)(ek[z] >> 32), (uint32_t)ek[z]);
        } else {
          et_has_n<EP>(a.g.etab, a.g.etbits, ek, ea, er);
        }
#pragma unroll
        for (int z = 0; z < EP; ++z) {
          if (q0 + z >= UN) break;
          etq += ea[z] ? 1 : 0;
          if (er[z]) c[q0 + z] |= HP_EXCL;
        }
      }
#pragma unroll
      for (int q = 0; q < UN; ++q) {
        if ((uint32_t)q >= nq) break;
        const bool valid = kq[q] != HP_EMPTY;
        if (!CUSTOM && !KD) drained += valid ? 1 : 0;  // deg w gathered for it
        const uint32_t sl = valid ? kq[q] >> wbits : 0u, w = kq[q] & wmask;
        const uint32_t uu = s_u[wv][sl];
        const uint64_t du2 = s_du[wv][sl];
        float s = 0.0f;
        if (valid) {
          if (CUSTOM) s = ho_score(c[q]);
          else s = score_basic(a.metric, (c[q] & HP_EXCL) ? 0u : (c[q] & (KD ? 1023u : HP_CMASK)), du2, (uint64_t)dw[q]);
        }
        hp_emit(sg, a, valid, s, uu, w, tau);
      }
    }
    wave_sync_lds();
    ph_mark(3);  // drain, scores, emission
    round = 0;  // every owner word of the batch is free again
    r0 = pr0;
    nr = pnr;
    u = pu;
    W = pW;
    s0 = ps0;
    ns = pns;
    o0 = po0;
    du = pdu;
    dx = pdx;
    b = bn;
  }
  hp_finish(sg, a, wedges);
  if (a.ph && lane == 0)
    for (int i = 0; i < 4; ++i) atomicAdd(&a.ph[i], (unsigned long long)ph_acc[i]);
  // + per wedge its key (and its degree for KD), per emitted candidate 16 (key, u, w, score)
  const uint64_t wsum = wave_sum(wedges);
  abytes += (KD ? 8ull : 4ull) * wsum + 16ull * sg.out + 4ull * wave_sum(drained) + 8ull * wave_sum(etq);
  if (lane == 0 && abytes) atomicAdd(&a.ctr[HPC_HOTB], (unsigned long long)abytes);
}

// ---------------------------------------------------------------- bins 1-3: workgroup per row
// GLOBAL = false: LDS table of up to HP_BT entries (HP_BT / 2 for AA / RA;
// bin 1).  GLOBAL = true: per-workgroup slab of 2^tlog entries in global memory
// (bins 2, 3); a row whose distinct-w bound exceeds the slab is split into
// w-range passes.
__device__ __forceinline__ uint64_t block_incl_scan_1024(uint64_t x, uint64_t* s_w /*16*/) {
  const uint64_t inc = wave_incl_scan(x);
  if (lane_id() == 63) s_w[wave_id()] = inc;
  __syncthreads();
  uint64_t pre = 0;
  for (int q = 0; q < wave_id(); ++q) pre += s_w[q];
  __syncthreads();
  return pre + inc;
}

constexpr int HP_BSTG = 128;  // staging per wave in the block kernels

// Workgroup barrier.  A global table is accessed with agent-scope atomics at
// L2, so the barrier must also wait for this wave's outstanding global
// operations (no-return atomics, the resets of the previous row): an
// agent-scope release/acquire around the barrier.
template <bool GLOBAL>
__device__ __forceinline__ void hp_sync() {
  if (GLOBAL) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (GLOBAL) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

template <bool CUSTOM, bool GLOBAL, bool KD = false>
__global__ __launch_bounds__(HP_BNT) void k_hp_block(HpArgs a, const uint32_t* __restrict__ rows, uint64_t nrows,
                                                     const uint64_t* __restrict__ wu, uint64_t ua,
                                                     uint32_t* __restrict__ slab, int tlog,
                                                     uint32_t* __restrict__ queue = nullptr) {
  constexpr int LT = GLOBAL ? 1 : (CUSTOM ? HP_BT / 2 : HP_BT);
  constexpr int VT = CUSTOM ? LT : 1;
  constexpr int NW = HP_BNT / 64;
  __shared__ uint32_t s_k[LT];
  __shared__ uint32_t s_c[LT];
  __shared__ uint32_t s_v0[VT];
  __shared__ uint32_t s_v1[VT];
  __shared__ uint64_t s_incl[HP_BNT];
  __shared__ uint64_t s_start[HP_BNT];
  __shared__ uint32_t s_iv[HP_BNT];
  __shared__ uint64_t s_w[NW];
  __shared__ uint64_t s_tot;
  __shared__ uint32_t s_gu[NW][HP_BSTG], s_gw[NW][HP_BSTG];
  __shared__ float s_gs[NW][HP_BSTG];
  __shared__ uint64_t s_it;
  // AA / RA in LDS: ordered accumulation (see ho_add_block) over S(u) sorted here
  constexpr bool ORD = CUSTOM && !GLOBAL;
  constexpr int SK = ORD ? LT / 2 : 1;
  __shared__ uint32_t s_sk[SK];
  __shared__ double s_ic[ORD ? HP_BNT : 1];
  const int t = threadIdx.x, wv = wave_id();
  const uint64_t tmax = GLOBAL ? (1ull << tlog) : (uint64_t)LT;
  HpTable tb;
  if (GLOBAL) {
    tb.k = slab + (uint64_t)blockIdx.x * tmax * 4;  // [keys | counts | vmin | vmax] per workgroup
    tb.c = tb.k + tmax;
    tb.vmin = tb.c + tmax;
    tb.vmax = tb.vmin + tmax;
  } else {
    tb = HpTable{s_k, s_c, s_v0, s_v1};
    for (int i = t; i < LT; i += HP_BNT) {
      s_k[i] = HP_EMPTY;
      s_c[i] = 0;
      if (CUSTOM) s_v0[i] = 0;  // owner tokens
    }
  }
  HpStage sg{s_gu[wv], s_gw[wv], s_gs[wv], HP_BSTG, 0, 0, 0};
  const int64_t tau = *a.tau;
  uint64_t wedges = 0;
  __syncthreads();
  // rows from a work queue when one is given (row costs vary), else a static stride
  for (uint64_t r0 = blockIdx.x;; r0 += gridDim.x) {
    uint64_t ri = r0;
    if (queue) {
      if (t == 0) s_it = atomicAdd(queue, 1u);
      __syncthreads();
      ri = s_it;
      __syncthreads();
    }
    if (ri >= nrows) break;
    const uint32_t u = rows[ri];
    const uint64_t W = wu[u - ua];
    const uint64_t o0 = a.g.off[u], o1 = a.g.off[u + 1];
    const uint64_t du = o1 - o0;
    const uint64_t span_w = a.S - 1 - u;              // candidate w in (u, S)
    const uint64_t need = 2 * (W < span_w ? W : span_w);
    const int tl = GLOBAL ? tlog : (CUSTOM ? 12 : 13);
    int lg = max(6, log2_ceil(need));
    uint64_t passes = 1;
    if (lg > tl) {
      // w-range passes no wider than half the table: at most tmax / 2 distinct w per pass
      passes = (2 * span_w + tmax - 1) / tmax;
      lg = tl;
    }
    const uint32_t T = 1u << lg, mask = T - 1;
    const int shift = 32 - lg;
    const uint64_t rw = (span_w + passes - 1) / passes;
    const uint32_t* fh;
    uint64_t nf;
    hp_first_hops(a, u, o0, du, &fh, &nf);
    if (ORD && a.soff && !a.ssorted) {  // S(u) from in-edge atomics is unordered: sort it
      if (nf > (uint64_t)SK) {
        if (t == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
        continue;  // uniform: nf is the workgroup's row
      }
      const uint32_t n2 = pow2_at_least((uint32_t)nf);
      for (uint32_t e = (uint32_t)t; e < n2; e += HP_BNT) s_sk[e] = e < nf ? fh[e] : 0xffffffffu;
      __syncthreads();
      block_bitonic_u32(s_sk, n2);
      fh = s_sk;
    }
    uint32_t round = 0;
    // packed survivor entries (the part of N(v) above u, no row-bound gather)
    const uint64_t* fd = a.sdo && a.soff && fh != (const uint32_t*)s_sk ? a.sdo + (fh - a.skeys) : nullptr;
    for (uint64_t p = 0; p < passes; ++p) {
      const uint64_t wlo = (uint64_t)u + 1 + p * rw;
      const uint64_t whi = wlo + rw < a.S ? wlo + rw : a.S;
      for (uint64_t base = 0; base < nf; base += HP_BNT) {
        const uint64_t i = base + t;
        uint32_t v = 0;
        uint64_t len = 0, st = 0;
        double cv = 0.0;
        if (i < nf) {
          if (fd) {
            const uint64_t x = fd[i];
            len = (uint32_t)(x >> HP_SDO_SH) & 0xffu;
            st = x & ((1ull << HP_SDO_SH) - 1);
            if (ORD) cv = a.g.ctab[x >> 48];
          } else {
            v = fh[i];
            const uint32_t d = a.g.deg[v];
            if (hp_surv(d, a.H)) {
              len = d;
              st = a.g.off[v];
              if (ORD) cv = a.g.ctab[d];
            }
          }
        }
        const uint64_t incl = block_incl_scan_1024(len, s_w);
        s_incl[t] = incl;
        s_start[t] = st;
        s_iv[t] = v;
        if (ORD) s_ic[t] = cv;
        if (t == HP_BNT - 1) s_tot = incl;
        hp_sync<GLOBAL>();
        const uint64_t total = s_tot;
        if constexpr (ORD) {
          hp_wedges<HP_BNT, true>(total, (uint32_t)t, (uint32_t)HP_BNT, s_incl, s_start, s_iv, a.g.keys,
                                  [&](bool ok, uint32_t w, uint32_t ent) {
                                    const bool in = ok && w > u && (uint64_t)w >= wlo && (uint64_t)w < whi;
                                    if (ok && w > u && p == 0) ++wedges;
                                    uint32_t h = 0;
                                    if (in) h = ho_find(tb, mask, shift, w, &a.ctr[HPC_ERR]);
                                    ho_add_block(tb, in, h, s_ic[ent], &round);
                                  });
        } else if constexpr (KD && !GLOBAL && !CUSTOM) {  // bin 1: W <= 4096, counts in 13 bits
          hp_wedges<HP_BNT, false, true>(total, (uint32_t)t, (uint32_t)HP_BNT, s_incl, s_start, s_iv, a.g.keys,
                                         [&](uint32_t w, uint32_t, uint32_t dw) {
                                           if (w > u) {
                                             if (p == 0) ++wedges;
                                             if ((uint64_t)w >= wlo && (uint64_t)w < whi)
                                               hp_insert_kd<13>(tb, mask, shift, w, dw, &a.ctr[HPC_ERR]);
                                           }
                                         }, a.kdeg);
        } else {
          hp_wedges<HP_BNT>(total, (uint32_t)t, (uint32_t)HP_BNT, s_incl, s_start, s_iv, a.g.keys,
                            [&](uint32_t w, uint32_t v) {
                              if (w > u) {
                                if (p == 0) ++wedges;
                                if ((uint64_t)w >= wlo && (uint64_t)w < whi)
                                  hp_insert<GLOBAL, CUSTOM>(tb, mask, shift, w, v, &a.ctr[HPC_ERR]);
                              }
                            });
        }
        hp_sync<GLOBAL>();
      }
      const uint32_t xu = a.xs ? a.xs[u] : 0u;  // the entries of N(u) above u
      // marked, or (LDS table, a slice beyond HB_XF times W) tested in the membership table at the drain
      const bool ux = !GLOBAL && hp_use_etab(a, du - xu, W);
      if (!ux)
        hp_stream(a.g.keys + o0 + xu, du - xu, (uint32_t)t, (uint32_t)HP_BNT, [&](uint32_t x) {
          if ((uint64_t)x >= wlo && (uint64_t)x < whi) hp_mark<GLOBAL>(tb, mask, shift, x);
        });
      hp_sync<GLOBAL>();
      hp_drain<GLOBAL, CUSTOM, HP_UN, ORD, (KD && !GLOBAL && !CUSTOM) ? 13 : 0>(tb, T, (uint32_t)t, (uint32_t)HP_BNT,
                                                                              sg, a, u, du, tau, ux);
      hp_sync<GLOBAL>();
      round = 0;
    }
  }
  hp_finish(sg, a, wedges);
}

// ---------------------------------------------------------------- bin 1, count metrics: tiered rows
// k_hp_block holds 110 KB of LDS (a 1024-thread workgroup, an 8192-entry
// two-array table): one row in flight per CU, and a bin-1 row is a chain of
// dependent loads (row bounds, survivor entries, N(v), N(u)).  Count metrics
// with entry degrees take bin 1 here instead: a 256-thread workgroup per row
// and a one-word table (key << 32 | count word, hp_insert_kd's layout with 13
// count bits) sized by the row's tier -- W+ <= 1024: 2048 entries, <= 2048:
// 4096, <= 4096: 8192 -- so five, three or two rows are in flight per CU.
constexpr int HP_RNT = 256;
constexpr uint64_t HP_RTIER0 = 1024, HP_RTIER1 = 2048;

template <int LT, int RNT = HP_RNT>  // RNT threads per row
__global__ __launch_bounds__(RNT) void k_hp_rowb(HpArgs a, const uint32_t* __restrict__ tl,
                                                    const uint32_t* __restrict__ tcnt, int tier,
                                                    const uint64_t* __restrict__ wu, uint64_t ua,
                                                    uint32_t* __restrict__ queue) {
  constexpr int NW = RNT / 64;
  constexpr int TLG = LT == 2048 ? 11 : LT == 4096 ? 12 : 13;
  static_assert((1 << TLG) == LT, "table sizes 2048, 4096, 8192");
  __shared__ uint64_t s_t[LT];
  __shared__ uint64_t s_incl[RNT];
  __shared__ uint64_t s_start[RNT];
  __shared__ uint32_t s_iv[RNT];
  __shared__ uint64_t s_w[NW];
  __shared__ uint64_t s_tot;
  __shared__ uint32_t s_tk[3];
  __shared__ uint32_t s_gu[NW][HP_BSTG], s_gw[NW][HP_BSTG];
  __shared__ float s_gs[NW][HP_BSTG];
  const int t = threadIdx.x, wv = wave_id();
  uint32_t rbase, nrows;  // this tier's rows: a region of the tier list (k_hp_tier)
  hb_region(tcnt, tier, tier, &rbase, &nrows);
  const uint32_t* rows = tl + rbase;
  if (nrows == 0) return;
  for (int i = t; i < LT; i += RNT) s_t[i] = HP_EMPTY64;
  HpStage sg{s_gu[wv], s_gw[wv], s_gs[wv], HP_BSTG, 0, 0, 0};
  const int64_t tau = *a.tau;
  uint64_t wedges = 0;
  // Rows from the work queue in a three-stage pipeline: while row `cur` runs,
  // the next row's data (its W+, bounds, exclusion start, survivor range) and
  // the row id of the one after are in flight, and a further ticket is drawn
  // (a workgroup barrier waits for LDS only), so a row pays no queue or row
  // data round trip of its own.
  struct RowInfo {
    uint32_t u;
    uint64_t W, o0, du, xu, s0, ns;
  };
  auto info = [&](bool ok, uint32_t uu) {
    RowInfo r{0u, 0, 0, 0, 0, 0, 0};
    if (!ok) return r;
    r.u = uu;
    r.W = wu[uu - ua];
    r.o0 = a.g.off[uu];
    r.du = a.g.off[uu + 1] - r.o0;
    r.xu = a.xs ? a.xs[uu] : 0u;
    r.s0 = a.soff ? a.soff[uu - a.sua] : 0ull;
    r.ns = a.soff ? hp_slen(a, uu, r.s0) : r.du;
    return r;
  };
  if (t == 0) {
    s_tk[0] = atomicAdd(queue, 1u);
    s_tk[1] = atomicAdd(queue, 1u);
    s_tk[2] = atomicAdd(queue, 1u);
  }
  __syncthreads();
  const uint64_t k0 = s_tk[0], k1 = s_tk[1];
  uint64_t cur = k0, nx = k1, nn = s_tk[2];
  RowInfo ci = info(k0 < nrows, k0 < nrows ? rows[k0] : 0u);
  uint32_t nxu = k1 < nrows ? rows[k1] : 0u;
  __syncthreads();
  while (cur < nrows) {
    const RowInfo ni = info(nx < nrows, nxu);  // in flight during this row
    const uint32_t nnu = nn < nrows ? rows[nn] : 0u;
    uint32_t tk = 0;
    if (t == 0) tk = atomicAdd(queue, 1u);
    const uint32_t u = ci.u;
    const uint64_t W = ci.W, o0 = ci.o0, du = ci.du;
    const uint64_t span_w = a.S - 1 - u;  // candidate w in (u, S)
    const int lg = max(6, log2_ceil(2 * (W < span_w ? W : span_w)));
    bool skip = false;
    if (lg > TLG) {  // a row beyond its tier (a binning bug): fail the call, never overrun LDS
      if (t == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
      skip = true;
    }
    const uint32_t T = 1u << (skip ? 6 : lg), mask = T - 1;
    const int shift = 32 - (skip ? 6 : lg);
    const uint32_t* fh = a.soff ? a.skeys + ci.s0 : a.g.keys + o0;
    const uint64_t nf = skip ? 0 : ci.ns;
    // packed survivor entries (the part of N(v) above u, no row-bound gather)
    const uint64_t* fd = a.sdo && a.soff ? a.sdo + (fh - a.skeys) : nullptr;
    for (uint64_t base = 0; base < nf; base += RNT) {
      const uint64_t i = base + t;
      uint64_t len = 0, st = 0;
      if (i < nf) {
        if (fd) {
          const uint64_t x = fd[i];
          len = (uint32_t)(x >> HP_SDO_SH) & 0xffu;
          st = x & ((1ull << HP_SDO_SH) - 1);
        } else {
          const uint32_t v = fh[i], d = a.g.deg[v];
          if (hp_surv(d, a.H)) {
            len = d;
            st = a.g.off[v];
          }
        }
      }
      const uint64_t incl = block_incl_scan_1024(len, s_w);
      s_incl[t] = incl;
      s_start[t] = st;
      s_iv[t] = 0u;
      if (t == RNT - 1) s_tot = incl;
      __syncthreads();
      hp_wedges<RNT, false, true>(s_tot, (uint32_t)t, (uint32_t)RNT, s_incl, s_start, s_iv, a.g.keys,
                                     [&](uint32_t w, uint32_t, uint32_t dw) {
                                       if (w > u) {
                                         ++wedges;
                                         h64_insert<13>(s_t, mask, shift, w, dw, &a.ctr[HPC_ERR]);
                                       }
                                     }, a.kdeg);
      __syncthreads();
    }
    // first-order exclusion: the entries of N(u) above u (a key <= u has no
    // entry) marked, or -- a slice beyond HB_XF times the row's wedge bound --
    // every entry tested in the membership table at the drain
    const uint64_t xu = skip ? du : ci.xu;
    const bool ux = hp_use_etab(a, du - xu, W);
    if (!ux)
      hp_stream(a.g.keys + o0 + xu, du - xu, (uint32_t)t, (uint32_t)RNT,
                [&](uint32_t x) { h64_mark(s_t, mask, shift, x); });
    __syncthreads();
    for (uint32_t i0 = 0; i0 < T; i0 += RNT * HP_UN) {  // T >= 64: uniform per wave
      uint32_t kq[HP_UN], c[HP_UN], dw[HP_UN];
#pragma unroll
      for (int q = 0; q < HP_UN; ++q) {
        const uint32_t i = i0 + (uint32_t)q * RNT + (uint32_t)t;
        kq[q] = HP_EMPTY;
        c[q] = 0;
        if (i < T) {
          const uint64_t x = s_t[i];
          kq[q] = (uint32_t)(x >> 32);
          c[q] = (uint32_t)x;
          if (kq[q] != HP_EMPTY) s_t[i] = HP_EMPTY64;
        }
      }
#pragma unroll
      for (int q = 0; q < HP_UN; ++q) dw[q] = kq[q] != HP_EMPTY ? hp_kd_deg<13>(a.g, c[q], kq[q]) : 0u;
      if (ux) {  // the membership table, both probes in flight
        uint64_t ek[HP_UN];
        bool ea[HP_UN], er[HP_UN];
#pragma unroll
        for (int q = 0; q < HP_UN; ++q) {
          ea[q] = kq[q] != HP_EMPTY;
          ek[q] = ea[q] ? ((uint64_t)u << 32 | kq[q]) : 0ull;
        }
        et_has_n<HP_UN>(a.g.etab, a.g.etbits, ek, ea, er);
#pragma unroll
        for (int q = 0; q < HP_UN; ++q)
          if (er[q]) c[q] |= HP_EXCL;
      }
#pragma unroll
      for (int q = 0; q < HP_UN; ++q) {
        const bool valid = kq[q] != HP_EMPTY;
        float sc = 0.0f;
        if (valid) sc = score_basic(a.metric, (c[q] & HP_EXCL) ? 0u : (c[q] & 8191u), du, (uint64_t)dw[q]);
        hp_emit(sg, a, valid, sc, u, kq[q], tau);
      }
    }
    __syncthreads();
    if (t == 0) s_tk[0] = tk;
    __syncthreads();
    cur = nx;
    nx = nn;
    nn = s_tk[0];
    ci = ni;
    nxu = nnu;
  }
  hp_finish(sg, a, wedges);
}

// The same tiers for AA / RA (custom bin 1: W+ <= 2048): an ordered table
// (ho_add_block's owner tokens over 256 threads) of 2048 or 4096 entries,
// S(u) in ascending v (the degree-class lists are sorted by construction).
template <int LT, int RNT = HP_RNT>  // RNT threads per row (a power of two)
__global__ __launch_bounds__(RNT) void k_hp_rowo(HpArgs a, const uint32_t* __restrict__ tl,
                                                    const uint32_t* __restrict__ tcnt, int tier,
                                                    const uint64_t* __restrict__ wu, uint64_t ua,
                                                    uint32_t* __restrict__ queue) {
  constexpr int NW = RNT / 64;
  static_assert(RNT == 128 || RNT == 256, "owner tokens of 7 or 8 thread bits");
  constexpr int TLG = LT == 2048 ? 11 : 12;
  static_assert((1 << TLG) == LT, "table sizes 2048, 4096");
  __shared__ uint32_t s_k[LT], s_c[LT], s_o[LT];  // keys, float accumulators, owner tokens
  __shared__ uint64_t s_incl[RNT];
  __shared__ uint64_t s_start[RNT];
  __shared__ uint32_t s_iv[RNT];
  __shared__ double s_ic[RNT];
  __shared__ uint64_t s_w[NW];
  __shared__ uint64_t s_tot, s_it;
  __shared__ uint32_t s_gu[NW][HP_BSTG], s_gw[NW][HP_BSTG];
  __shared__ float s_gs[NW][HP_BSTG];
  const int t = threadIdx.x, wv = wave_id();
  uint32_t rbase, nrows;  // this tier's rows: a region of the tier list (k_hp_tier)
  hb_region(tcnt, tier, tier, &rbase, &nrows);
  const uint32_t* rows = tl + rbase;
  if (nrows == 0) return;
  const HpTable tb{s_k, s_c, s_o, s_o};
  for (int i = t; i < LT; i += RNT) {
    s_k[i] = HP_EMPTY;
    s_c[i] = 0;
    s_o[i] = 0;
  }
  HpStage sg{s_gu[wv], s_gw[wv], s_gs[wv], HP_BSTG, 0, 0, 0};
  const int64_t tau = *a.tau;
  uint64_t wedges = 0;
  __syncthreads();
  for (;;) {
    if (t == 0) s_it = atomicAdd(queue, 1u);
    __syncthreads();
    const uint64_t ri = s_it;
    __syncthreads();
    if (ri >= nrows) break;
    const uint32_t u = rows[ri];
    const uint64_t W = wu[u - ua];
    const uint64_t o0 = a.g.off[u], du = a.g.off[u + 1] - o0;
    const uint64_t span_w = a.S - 1 - u;
    const int lg = max(6, log2_ceil(2 * (W < span_w ? W : span_w)));
    if (lg > TLG) {  // a row beyond its tier (a binning bug): fail the call, never overrun LDS
      if (t == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
      continue;
    }
    const uint32_t T = 1u << lg, mask = T - 1;
    const int shift = 32 - lg;
    const uint32_t* fh;
    uint64_t nf;
    hp_first_hops(a, u, o0, du, &fh, &nf);
    const uint64_t* fd = a.sdo + (fh - a.skeys);  // packed survivor entries (host: sdo and sorted lists)
    uint32_t round = 0;
    for (uint64_t base = 0; base < nf; base += RNT) {
      const uint64_t i = base + t;
      uint64_t len = 0, st = 0;
      double cv = 0.0;
      if (i < nf) {
        const uint64_t x = fd[i];
        len = (uint32_t)(x >> HP_SDO_SH) & 0xffu;
        st = x & ((1ull << HP_SDO_SH) - 1);
        cv = a.g.ctab[x >> 48];
      }
      const uint64_t incl = block_incl_scan_1024(len, s_w);
      s_incl[t] = incl;
      s_start[t] = st;
      s_iv[t] = 0u;
      s_ic[t] = cv;
      if (t == RNT - 1) s_tot = incl;
      __syncthreads();
      // wedges in steps of one per thread, j ascending in the thread index:
      // the additions of each w in the reference's order of v (predict.hxx:788, 828)
      hp_wedges<RNT, true>(s_tot, (uint32_t)t, (uint32_t)RNT, s_incl, s_start, s_iv, a.g.keys,
                              [&](bool ok, uint32_t w, uint32_t ent) {
                                const bool in = ok && w > u;
                                if (in) ++wedges;
                                uint32_t h = 0;
                                if (in) h = ho_find(tb, mask, shift, w, &a.ctr[HPC_ERR]);
                                ho_add_block<RNT == 128 ? 7 : 8>(tb, in, h, s_ic[ent], &round);
                              });
      __syncthreads();
    }
    const uint32_t xu = a.xs ? a.xs[u] : 0u;
    const bool ux = hp_use_etab(a, du - xu, W);
    if (!ux)
      hp_stream(a.g.keys + o0 + xu, du - xu, (uint32_t)t, (uint32_t)RNT,
                [&](uint32_t x) { hp_mark<false>(tb, mask, shift, x); });
    __syncthreads();
    hp_drain<false, true, HP_UN, true, 0>(tb, T, (uint32_t)t, (uint32_t)RNT, sg, a, u, du, tau, ux);
    __syncthreads();  // (ho_take reset every used entry's owner token)
  }
  hp_finish(sg, a, wedges);
}

// ---------------------------------------------------------------- bins 2-3: partitioned rows
// A row whose wedges overflow an LDS table is cut into P w-buckets of width
// 2^shift (P <= HP_PMAX).  Pass A counts the row's wedges per bucket (LDS
// histogram), pass B scatters them bucket by bucket into the workgroup's
// scratch (w, and v for AA / RA), and every bucket is then accumulated in the
// LDS table from its contiguous scratch range -- one streaming write and read
// of the wedges instead of two global atomics each.  Buckets are processed in
// ascending w, so the first-order exclusion walks N(u) with a single cursor.
// Groups of buckets are formed so that a group's wedges fit the scratch; a
// single bucket beyond the scratch is accumulated directly from the row
// enumeration (rare: hub-hub concentrations).
constexpr int HP_PMAX = 4096;
constexpr uint64_t HP_PART_W = 1024;  // wedges per w-bucket

// Row expansion shared by the passes: calls f(w, v) for every wedge (u, v, w)
// with w > u, v surviving; every thread of the workgroup must call it.
// With a w-range [wlo, whi) (a row slice of k_hp_part) each list N(v) is cut to
// that range by two binary searches (lists are sorted), so a slice enumerates
// only its own wedges; wlo = 0 enumerates whole lists.
template <typename F>
__device__ __forceinline__ void hp_enum_row(const HpArgs& a, uint32_t u, uint64_t o0, uint64_t du, uint64_t* s_incl,
                                            uint64_t* s_start, uint32_t* s_iv, uint64_t* s_w, uint64_t* s_tot, F f,
                                            uint64_t wlo = 0, uint64_t whi = 0) {
  const int t = threadIdx.x;
  const uint32_t* fh;
  uint64_t nf;
  hp_first_hops(a, u, o0, du, &fh, &nf);
  for (uint64_t base = 0; base < nf; base += HP_BNT) {
    const uint64_t i = base + t;
    uint32_t v = 0;
    uint64_t len = 0, st = 0;
    if (i < nf) {
      v = fh[i];
      const uint32_t d = a.g.deg[v];
      if (hp_surv(d, a.H)) {
        len = d;
        st = a.g.off[v];
        if (wlo) {
          const uint32_t* L = a.g.keys + st;
          uint32_t l = 0, h = d;
          while (l < h) {
            const uint32_t m = (l + h) >> 1;
            if ((uint64_t)L[m] < wlo) l = m + 1; else h = m;
          }
          uint32_t e = l, h2 = d;
          while (e < h2) {
            const uint32_t m = (e + h2) >> 1;
            if ((uint64_t)L[m] < whi) e = m + 1; else h2 = m;
          }
          st += l;
          len = e - l;
        }
      }
    }
    const uint64_t incl = block_incl_scan_1024(len, s_w);
    s_incl[t] = incl;
    s_start[t] = st;
    s_iv[t] = v;
    if (t == HP_BNT - 1) *s_tot = incl;
    __syncthreads();
    const uint64_t total = *s_tot;
    hp_wedges<HP_BNT>(total, (uint32_t)t, (uint32_t)HP_BNT, s_incl, s_start, s_iv, a.g.keys,
                      [&](uint32_t w, uint32_t v) {
                        if (w > u) f(w, v);
                      });
    __syncthreads();
  }
}

// exclusive scan of s[0..n) in place (n <= HP_PMAX)
__device__ __forceinline__ void hp_scan_buckets(uint32_t* s, uint32_t n, uint64_t* s_w) {
  constexpr int PER = HP_PMAX / HP_BNT;
  const int t = threadIdx.x;
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint32_t i = (uint32_t)t * PER + q;
    v[q] = i < n ? s[i] : 0u;
    sum += v[q];
  }
  const uint64_t incl = block_incl_scan_1024(sum, s_w);
  uint32_t run = (uint32_t)(incl - sum);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint32_t i = (uint32_t)t * PER + q;
    if (i < n) s[i] = run;
    run += v[q];
  }
  __syncthreads();
}

template <bool CUSTOM>
__global__ __launch_bounds__(HP_BNT) void k_hp_part(HpArgs a, const uint32_t* __restrict__ rows, uint64_t nrows,
                                                    const uint64_t* __restrict__ wu, uint64_t ua,
                                                    uint32_t* __restrict__ scratch, uint64_t scap, uint32_t nsl,
                                                    uint32_t* __restrict__ queue) {
  constexpr int LT = CUSTOM ? HP_BT / 2 : HP_BT;
  constexpr int VT = CUSTOM ? LT : 1;
  constexpr int NW = HP_BNT / 64;
  constexpr int TL = CUSTOM ? 12 : 13;
  __shared__ uint32_t s_k[LT];
  __shared__ uint32_t s_c[LT];
  __shared__ uint32_t s_v0[VT];
  __shared__ uint32_t s_v1[VT];
  __shared__ uint64_t s_incl[HP_BNT];
  __shared__ uint64_t s_start[HP_BNT];
  __shared__ uint32_t s_iv[HP_BNT];
  __shared__ uint64_t s_w[NW];
  __shared__ uint64_t s_tot;
  __shared__ uint32_t s_bc[HP_PMAX];   // wedges per bucket
  __shared__ uint32_t s_bo[HP_PMAX];   // scratch offset per bucket (group-relative), then scatter cursor
  __shared__ uint32_t s_g1, s_gdirect, s_xcur;
  __shared__ uint64_t s_it;
  __shared__ uint32_t s_gu[NW][HP_BSTG], s_gw[NW][HP_BSTG];
  __shared__ float s_gs[NW][HP_BSTG];
  const int t = threadIdx.x, wv = wave_id();
  const HpTable tb{s_k, s_c, s_v0, s_v1};
  for (int i = t; i < LT; i += HP_BNT) {
    s_k[i] = HP_EMPTY;
    s_c[i] = 0;
    if (CUSTOM) { s_v0[i] = HP_EMPTY; s_v1[i] = 0; }
  }
  uint32_t* sw = scratch + (uint64_t)blockIdx.x * scap * (CUSTOM ? 2 : 1);
  uint32_t* sv = sw + scap;
  HpStage sg{s_gu[wv], s_gw[wv], s_gs[wv], HP_BSTG, 0, 0, 0};
  const int64_t tau = *a.tau;
  uint64_t wedges = 0;
  __syncthreads();
  // Work items are (row, slice): slice sl of a row owns buckets
  // [P sl / nsl, P (sl + 1) / nsl), so that a few huge rows (bin 3) spread
  // over many workgroups instead of holding one CU each while the chip idles.
  // Every slice enumerates the whole row (the lists are hot in L2) and keeps
  // only its buckets' wedges.  Items are taken from a work queue (one atomic
  // per item): row costs vary by orders of magnitude, and a static stride left
  // a few workgroups with the heavy rows.
  const uint64_t nit = nrows * nsl;
  for (;;) {
    if (t == 0) s_it = atomicAdd(queue, 1u);
    __syncthreads();
    const uint64_t it = s_it;
    __syncthreads();
    if (it >= nit) break;
    const uint64_t ri = it / nsl;
    const uint32_t sl = (uint32_t)(it - ri * nsl);
    const uint32_t u = rows[ri];
    const uint64_t W = wu[u - ua];
    const uint64_t o0 = a.g.off[u], du = a.g.off[u + 1] - o0;
    const uint64_t span_w = a.S - 1 - u;  // candidate w in (u, S)
    if (span_w == 0) continue;
    // buckets: about HP_PART_W wedges each, never narrower than needed
    uint64_t pd = (W + HP_PART_W - 1) / HP_PART_W;
    const uint64_t pspan = (span_w + (LT / 2) - 1) / (LT / 2);
    if (pd > pspan) pd = pspan;
    if (pd < 1) pd = 1;
    if (pd > HP_PMAX) pd = HP_PMAX;
    const int shift = log2_ceil((span_w + pd - 1) / pd);
    const uint32_t P = (uint32_t)((span_w + (1ull << shift) - 1) >> shift);
    const uint32_t bs0 = (uint32_t)((uint64_t)P * sl / nsl), bs1 = (uint32_t)((uint64_t)P * (sl + 1) / nsl);
    if (bs0 == bs1) continue;  // an empty slice (uniform across the workgroup)
    // w-range of the slice for the enumeration (0: whole lists when the row is not sliced)
    const uint64_t slo0 = nsl > 1 ? (uint64_t)u + 1 + ((uint64_t)bs0 << shift) : 0;
    const uint64_t shi0 = nsl > 1 ? std::min<uint64_t>(a.S, (uint64_t)u + 1 + ((uint64_t)bs1 << shift)) : 0;
    for (uint32_t b = t; b < P; b += HP_BNT) s_bc[b] = 0;
    if (t == 0) {  // exclusion cursor: first entry of N(u) in the slice, i.e. >= u + 1 + (bs0 << shift)
      const uint64_t x0 = (uint64_t)u + 1 + ((uint64_t)bs0 << shift);
      uint64_t lo = 0, hi = du;
      while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if ((uint64_t)a.g.keys[o0 + m] < x0) lo = m + 1; else hi = m;
      }
      s_xcur = (uint32_t)lo;
    }
    __syncthreads();
    // pass A: wedges per bucket of the slice
    hp_enum_row(a, u, o0, du, s_incl, s_start, s_iv, s_w, &s_tot, [&](uint32_t w, uint32_t) {
      const uint32_t b = (w - u - 1) >> shift;
      if (b >= bs0 && b < bs1) {
        ++wedges;
        atomicAdd(&s_bc[b], 1u);
      }
    }, slo0, shi0);
    for (uint32_t b0 = bs0; b0 < bs1;) {
      if (t == 0) {
        uint64_t sum = 0;
        uint32_t b = b0;
        while (b < bs1 && sum + s_bc[b] <= scap) sum += s_bc[b++];
        s_gdirect = b == b0 ? 1u : 0u;
        s_g1 = b == b0 ? b0 + 1 : b;
      }
      __syncthreads();
      const uint32_t b1 = s_g1;
      const bool direct = s_gdirect != 0;
      if (!direct) {
        // group offsets and pass B: scatter the group's wedges bucket by bucket
        for (uint32_t b = t; b < b1 - b0; b += HP_BNT) s_bo[b] = s_bc[b0 + b];
        __syncthreads();
        hp_scan_buckets(s_bo, b1 - b0, s_w);
        hp_enum_row(a, u, o0, du, s_incl, s_start, s_iv, s_w, &s_tot, [&](uint32_t w, uint32_t v) {
          const uint32_t b = (w - u - 1) >> shift;
          if (b >= b0 && b < b1) {
            const uint32_t p = atomicAdd(&s_bo[b - b0], 1u);
            sw[p] = w;
            if (CUSTOM) sv[p] = v;
          }
        }, slo0, shi0);
        hp_sync<true>();
      }
      // buckets of the group, ascending w
      uint32_t boff = 0;
      for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t nb = s_bc[b];
        const uint32_t off = boff;
        boff += nb;
        if (nb == 0) continue;
        const uint64_t lo = (uint64_t)u + 1 + ((uint64_t)b << shift);
        const uint64_t hi = lo + (1ull << shift) < a.S ? lo + (1ull << shift) : a.S;
        const uint64_t width = hi - lo;
        const uint64_t need = 2 * ((uint64_t)nb < width ? (uint64_t)nb : width);
        int lg = max(6, log2_ceil(need));
        uint64_t sub = 1;
        if (lg > TL) {
          sub = (2 * width + (1ull << TL) - 1) >> TL;
          lg = TL;
        }
        const uint32_t T = 1u << lg, mask = T - 1;
        const int hs = 32 - lg;
        const uint64_t sw_w = (width + sub - 1) / sub;
        for (uint64_t q = 0; q < sub; ++q) {
          const uint64_t slo = lo + q * sw_w;
          const uint64_t shi = slo + sw_w < hi ? slo + sw_w : hi;
          if (!direct) {
            for (uint32_t i0 = 0; i0 < nb; i0 += HP_BNT * HP_UN) {  // HP_UN scratch words per lane in flight
              uint32_t wq[HP_UN], vq[HP_UN];
#pragma unroll
              for (int r = 0; r < HP_UN; ++r) {
                const uint32_t i = i0 + (uint32_t)r * HP_BNT + (uint32_t)t;
                const uint32_t ii = i < nb ? i : 0u;
                wq[r] = sw[off + ii];
                vq[r] = CUSTOM ? sv[off + ii] : 0u;
              }
#pragma unroll
              for (int r = 0; r < HP_UN; ++r) {
                const uint32_t i = i0 + (uint32_t)r * HP_BNT + (uint32_t)t;
                if (i < nb && (sub == 1 || ((uint64_t)wq[r] >= slo && (uint64_t)wq[r] < shi)))
                  hp_insert<false, CUSTOM>(tb, mask, hs, wq[r], vq[r], &a.ctr[HPC_ERR]);
              }
            }
            __syncthreads();
          } else {
            hp_enum_row(a, u, o0, du, s_incl, s_start, s_iv, s_w, &s_tot, [&](uint32_t w, uint32_t v) {
              if ((uint64_t)w >= slo && (uint64_t)w < shi) hp_insert<false, CUSTOM>(tb, mask, hs, w, v, &a.ctr[HPC_ERR]);
            }, slo, shi);
          }
          // first-order exclusion: the entries of N(u) in [slo, shi) (cursor walk)
          for (;;) {
            const uint32_t xc = s_xcur;
            const uint64_t i = (uint64_t)xc + t;
            bool in = false;
            if (i < du) {
              const uint32_t x = a.g.keys[o0 + i];
              in = (uint64_t)x < shi;
              if (in) hp_mark<false>(tb, mask, hs, x);
            }
            const uint64_t m = __ballot(in);
            if (lane_id() == 0) s_w[wv] = (uint64_t)__popcll(m);
            __syncthreads();
            uint32_t adv = 0;
            for (int q2 = 0; q2 < NW; ++q2) adv += (uint32_t)s_w[q2];
            __syncthreads();
            if (t == 0) s_xcur = xc + adv;
            __syncthreads();
            if (adv < HP_BNT) break;
          }
          __syncthreads();
          hp_drain<false, CUSTOM>(tb, T, (uint32_t)t, (uint32_t)HP_BNT, sg, a, u, du, tau);
          __syncthreads();
        }
      }
      b0 = b1;
    }
    __syncthreads();  // the next row rewrites s_bc / s_xcur
  }
  hp_finish(sg, a, wedges);
}

// ---------------------------------------------------------------- bins 2-3: the hub pass
// k_hp_part works a hub row's w-buckets one after another on one workgroup
// (the few largest rows of a chunk then run on a handful of CUs), and a sliced
// row makes every slice walk the whole first-hop list.  The hub pass instead
// spreads both halves of the work over the chip:
//   k_hh_rows     per hub row: its w-bucket width (about HH_BW of W(u) per
//                 bucket, at most HH_PMAX buckets) and its enumeration items
//                 (HH_WC wedges of the row's flattened first-hop lists each: a
//                 row of an IHub call may hold a few first hops with millions
//                 of wedges -- items by first hops left one workgroup per row);
//   k_hh_fpre     per hub row the inclusive prefix of its first hops' lengths
//                 (an item finds its first first hop by binary search);
//   k_hh_maps     bucket -> row, and every bucket's first entry of N(u) (the
//                 exclusion slice, one binary search per bucket);
//   k_hh_enum     one workgroup per item (its row by binary search of the item
//                 prefix): its wedges counted per bucket in LDS and added to the
//                 global bucket counts (COUNT); then, after a scan, counted
//                 again, reserved with one atomic per used bucket and written to
//                 the bucket's contiguous scratch (SCATTER: w, and v for AA /
//                 RA).  Consecutive lanes take consecutive entries of a sorted
//                 list N(v), so equal buckets come in runs: one LDS atomic per
//                 run of a wave (its head lane), not per wedge;
//   k_hh_accum    one workgroup per bucket (work queue): its wedges into an
//                 LDS table, the exclusion slice of N(u) marked, every entry
//                 scored and emitted -- buckets of different rows in parallel.
// A bucket whose distinct-w bound exceeds the table is accumulated in w-range
// sub-passes over its scratch.  When a chunk's hub wedges exceed the scratch
// the host keeps k_hp_part for that chunk.
constexpr uint64_t HH_BW = 1024;    // W(u) per w-bucket (W counts every w, so buckets hold at most about this)
constexpr uint32_t HH_PMAX = 8192;  // buckets per row at most
constexpr uint64_t HH_WC = 16384;   // wedges (every w of the row's flattened lists) per enumeration item
constexpr int HH_NT = 256;          // threads of the enumeration and accumulation workgroups
constexpr int HH_NW = HH_NT / 64;
constexpr int HH_TL = 13;           // accumulation table: 2^13 LDS entries (2^12 for AA / RA)
constexpr int HH_XP = 2;            // exclusion keys per thread loaded with an item's first wedges
constexpr int HH_TLC = 12;          // the count metrics' default table log (k_hh_accum<false, 12>)
constexpr int HH_AUN = 8;           // an item's wedges per thread loaded together (most items: one round trip)

__device__ __forceinline__ uint32_t hh_row_u(const uint32_t* l2, uint64_t n2, const uint32_t* l3, uint64_t r) {
  return r < n2 ? l2[r] : l3[r - n2];
}

__global__ void k_hh_rows(HpArgs a, const uint32_t* __restrict__ l2, uint64_t n2, const uint32_t* __restrict__ l3,
                          uint64_t n3, const uint64_t* __restrict__ wu, uint64_t ua, uint32_t* __restrict__ hr_u,
                          uint32_t* __restrict__ hr_shift, uint32_t* __restrict__ hr_p, uint32_t* __restrict__ hr_items,
                          uint64_t* __restrict__ hr_nf, uint64_t bw = HH_BW) {
  const uint64_t nh = n2 + n3;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nh; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = hh_row_u(l2, n2, l3, r);
    const uint64_t W = wu[u - ua];
    const uint64_t span_w = a.S - 1 - u;  // candidate w in (u, S)
    uint64_t nf = 0;
    if (span_w > 0 && W > 0) {
      if (a.soff) nf = hp_slen(a, u, a.soff[u - a.sua]);
      else nf = a.g.off[u + 1] - a.g.off[u];
    }
    hr_u[r] = u;
    hr_nf[r] = nf;
    (void)hr_shift;
    (void)hr_p;
    (void)hr_items;
    (void)bw;
  }
}

// After k_hh_fpre: per hub row its wedges above u, Wr = the last inclusive
// prefix of its first hops' above-u lengths, give the w-buckets (about bw
// wedges each, at most HH_PMAX) and the enumeration items (HH_WC wedges each)
// -- sized by the wedges the row really enumerates, not by W(u) (every w).
__global__ void k_hh_items(HpArgs a, uint64_t nh, const uint32_t* __restrict__ hr_u, const uint64_t* __restrict__ hr_nf,
                           const uint64_t* __restrict__ fbase, const uint64_t* __restrict__ fp,
                           uint32_t* __restrict__ hr_shift, uint32_t* __restrict__ hr_p, uint32_t* __restrict__ hr_items,
                           uint64_t bw) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nh; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = hr_u[r];
    const uint64_t nf = hr_nf[r];
    const uint64_t Wr = nf ? fp[fbase[r] + nf - 1] : 0ull;
    const uint64_t span_w = a.S - 1 - u;
    uint32_t P = 0, shift = 0, items = 0;
    if (Wr > 0 && span_w > 0) {
      uint64_t pd = (Wr + bw - 1) / bw;
      if (pd < 1) pd = 1;
      if (pd > HH_PMAX) pd = HH_PMAX;
      shift = (uint32_t)log2_ceil((span_w + pd - 1) / pd);
      P = (uint32_t)((span_w + (1ull << shift) - 1) >> shift);
      items = (uint32_t)std::min<uint64_t>((Wr + HH_WC - 1) / HH_WC, 0x7fffffffull);
    }
    hr_shift[r] = shift;
    hr_p[r] = P;
    hr_items[r] = items;
  }
}

// brow[bucket] = row, irow[item] = row, xs[bucket] = the first entry of N(u)
// at or above the bucket's w-range start (absolute index into keys)
__global__ void k_hh_maps(HpArgs a, uint64_t nh, const uint32_t* __restrict__ hr_u,
                          const uint32_t* __restrict__ hr_shift, const uint32_t* __restrict__ hr_p,
                          const uint64_t* __restrict__ bbase, const uint32_t* __restrict__ hr_items,
                          const uint64_t* __restrict__ ibase, uint32_t* __restrict__ brow, uint32_t* __restrict__ irow) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nh; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b0 = bbase[r], i0 = ibase[r];
    for (uint32_t b = 0; b < hr_p[r]; ++b) brow[b0 + b] = (uint32_t)r;
    (void)i0;
  }
}

__global__ void k_hh_xstart(HpArgs a, uint64_t nb, const uint32_t* __restrict__ brow, const uint32_t* __restrict__ hr_u,
                            const uint32_t* __restrict__ hr_shift, const uint64_t* __restrict__ bbase,
                            uint64_t* __restrict__ xs) {
  for (uint64_t gb = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; gb < nb; gb += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = brow[gb];
    const uint32_t u = hr_u[r];
    const uint64_t b = gb - bbase[r];
    const uint64_t x0 = (uint64_t)u + 1 + (b << hr_shift[r]);
    const uint64_t o0 = a.g.off[u];
    uint32_t n = (uint32_t)(a.g.off[u + 1] - o0);
    xs[gb] = o0 + (x0 > 0xffffffffull ? n : upper_bound_u32(a.g.keys + o0, n, (uint32_t)(x0 - 1)));
  }
}

// The row's first hops and the lengths of their lists in the flattened wedge
// space: S(u) with the packed entries (the part of N(v) above u), else the
// first hops with their whole lists when they survive the hub filter.
struct HhHops {
  const uint32_t* fh;
  const uint64_t* fd;
  uint64_t nf;
};
__device__ __forceinline__ HhHops hh_hops(const HpArgs& a, uint32_t u) {
  HhHops h;
  hp_first_hops(a, u, a.g.off[u], a.g.off[u + 1] - a.g.off[u], &h.fh, &h.nf);
  h.fd = a.sdo && a.soff ? a.sdo + (h.fh - a.skeys) : nullptr;
  return h;
}
// First hop i of row u: v, and the part of N(v) above u, [st, st + len) --
// only w > u are candidates (predict.hxx:221), and N(v) is sorted, so the
// entries at or below u are a prefix: one binary search per first hop (none
// when N(v) starts above u) instead of enumerating wedges that are dropped.
// (The late rows of an IHub call see mostly w < u: the C5 shards of the
// highest ids enumerated three times their wedges before round 5.)
__device__ __forceinline__ void hh_hop(const HpArgs& a, const HhHops& h, uint32_t u, uint64_t i, uint32_t* v,
                                       uint64_t* st, uint64_t* len) {
  *v = h.fh[i];
  if (h.fd) {
    const uint64_t x = h.fd[i];
    *len = (uint32_t)(x >> HP_SDO_SH) & 0xffu;
    *st = x & ((1ull << HP_SDO_SH) - 1);
  } else {
    const uint32_t d = a.g.deg[*v];
    uint64_t lo = 0, hi = 0;
    if (hp_surv(d, a.H)) {
      lo = a.g.off[*v];
      hi = lo + d;
      if (a.g.keys[lo] <= u) {  // first entry above u
        uint64_t l = lo + 1, r = hi;
        while (l < r) {
          const uint64_t m = (l + r) >> 1;
          if (a.g.keys[m] <= u) l = m + 1; else r = m;
        }
        lo = l;
      }
    }
    *st = lo;
    *len = hi - lo;
  }
}

// fp[fbase[r] + i] = the inclusive prefix of the list lengths of row r's first hops (one workgroup per row)
__global__ __launch_bounds__(HH_NT) void k_hh_fpre(HpArgs a, uint64_t nh, const uint32_t* __restrict__ hr_u,
                                                   const uint64_t* __restrict__ hr_nf, const uint64_t* __restrict__ fbase,
                                                   uint64_t* __restrict__ fp) {
  __shared__ uint64_t s_w[HH_NW];
  __shared__ uint64_t s_tot;
  const int t = threadIdx.x;
  for (uint64_t r = blockIdx.x; r < nh; r += gridDim.x) {
    const uint64_t nf = hr_nf[r];
    if (nf == 0) continue;  // uniform
    const HhHops h = hh_hops(a, hr_u[r]);
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nf; b0 += HH_NT) {
      const uint64_t i = b0 + t;
      uint32_t v;
      uint64_t st, len = 0;
      if (i < nf) hh_hop(a, h, hr_u[r], i, &v, &st, &len);
      const uint64_t incl = block_incl_scan_1024(len, s_w);
      if (i < nf) fp[fbase[r] + i] = carry + incl;
      if (t == HH_NT - 1) s_tot = incl;
      __syncthreads();
      carry += s_tot;
      __syncthreads();
    }
  }
}

// The wedges (w > u) of item `item`: flattened positions [j0, j1) of the row's
// lists; f(b, w, v) on every thread of the workgroup (wave-convergent), b = the
// wedge's bucket or HH_NOB (no wedge on this lane).
constexpr uint32_t HH_NOB = 0xffffffffu;
constexpr int HH_UN = 4;
template <typename F>
__device__ __forceinline__ void hh_enum_range(const HpArgs& a, uint32_t u, uint32_t shift, const HhHops& h,
                                              const uint64_t* fpr, uint64_t f, uint64_t j0, uint64_t j1,
                                              uint64_t* s_incl, uint64_t* s_start, uint32_t* s_iv, uint64_t* s_w,
                                              uint64_t* s_tot, F fn) {
  const int t = threadIdx.x;
  for (uint64_t g0 = f; g0 < h.nf; g0 += HH_NT) {
    const uint64_t i = g0 + t;
    uint32_t v = 0;
    uint64_t st = 0, len = 0;
    if (i < h.nf) {
      const uint64_t e = fpr[i], s0 = i ? fpr[i - 1] : 0ull;
      const uint64_t lo = s0 > j0 ? s0 : j0, hi = e < j1 ? e : j1;
      if (hi > lo) {
        uint64_t full;
        hh_hop(a, h, u, i, &v, &st, &full);
        st += lo - s0;
        len = hi - lo;
      }
    }
    const uint64_t incl = block_incl_scan_1024(len, s_w);
    s_incl[t] = incl;
    s_start[t] = st;
    s_iv[t] = v;
    if (t == HH_NT - 1) *s_tot = incl;
    __syncthreads();
    const uint64_t total = *s_tot;
    for (uint64_t jb = 0; jb < total; jb += (uint64_t)HH_NT * HH_UN) {
      uint32_t w[HH_UN], vv[HH_UN];
      bool ok[HH_UN];
#pragma unroll
      for (int q = 0; q < HH_UN; ++q) {
        const uint64_t j = jb + (uint64_t)q * HH_NT + t;
        ok[q] = j < total;
        uint32_t lo = 0, hi = HH_NT - 1;  // first entry whose inclusive prefix exceeds j
        while (lo < hi) {
          const uint32_t m = (lo + hi) >> 1;
          if (s_incl[m] > j) hi = m; else lo = m + 1;
        }
        const uint64_t ex = lo ? s_incl[lo - 1] : 0ull;
        vv[q] = s_iv[lo];
        w[q] = ok[q] ? a.g.keys[s_start[lo] + (j - ex)] : 0u;
      }
#pragma unroll
      for (int q = 0; q < HH_UN; ++q) {
        const bool in = ok[q] && w[q] > u;
        fn(in ? (w[q] - u - 1) >> shift : HH_NOB, w[q], vv[q]);
      }
    }
    __syncthreads();
    // done when this block reached the item's end (uniform)
    if (g0 + HH_NT >= h.nf || fpr[g0 + HH_NT - 1] >= j1) break;
  }
}

template <bool SCATTER, bool CUSTOM>
__global__ __launch_bounds__(HH_NT) void k_hh_enum(HpArgs a, uint64_t nh, const uint32_t* __restrict__ hr_u,
                                                   const uint32_t* __restrict__ hr_shift,
                                                   const uint32_t* __restrict__ hr_p, const uint64_t* __restrict__ bbase,
                                                   const uint64_t* __restrict__ ibase,
                                                   const uint64_t* __restrict__ fbase, const uint64_t* __restrict__ fp,
                                                   uint32_t* __restrict__ bcnt, const uint64_t* __restrict__ boff,
                                                   uint32_t* __restrict__ bcur, uint32_t* __restrict__ sw,
                                                   uint32_t* __restrict__ sv) {
  __shared__ uint32_t s_h[HH_PMAX];
  __shared__ uint64_t s_incl[HH_NT], s_start[HH_NT];
  __shared__ uint32_t s_iv[HH_NT];
  __shared__ uint64_t s_w[HH_NW];
  __shared__ uint64_t s_tot, s_f;
  __shared__ uint32_t s_r;
  const int t = threadIdx.x, lane = lane_id();
  const uint64_t item = blockIdx.x;
  if (t == 0) {  // the item's row: the last r with ibase[r] <= item
    uint64_t lo = 0, hi = nh;
    while (hi - lo > 1) {
      const uint64_t m = (lo + hi) >> 1;
      if (ibase[m] <= item) lo = m; else hi = m;
    }
    s_r = (uint32_t)lo;
  }
  __syncthreads();
  const uint32_t r = s_r;
  const uint32_t u = hr_u[r], shift = hr_shift[r], P = hr_p[r];
  const uint64_t bb = bbase[r];
  const HhHops h = hh_hops(a, u);
  const uint64_t* fpr = fp + fbase[r];
  const uint64_t Wr = fpr[h.nf - 1];
  const uint64_t j0 = (item - ibase[r]) * HH_WC, j1 = j0 + HH_WC < Wr ? j0 + HH_WC : Wr;
  if (t == 0) {  // the first first hop whose list reaches past j0
    uint64_t lo = 0, hi = h.nf - 1;
    while (lo < hi) {
      const uint64_t m = (lo + hi) >> 1;
      if (fpr[m] > j0) hi = m; else lo = m + 1;
    }
    s_f = lo;
  }
  for (uint32_t b = t; b < P; b += HH_NT) s_h[b] = 0;
  __syncthreads();
  const uint64_t f = s_f;
  // a run of equal buckets over consecutive lanes: its head adds the run's length
  auto count = [&](uint32_t b, uint32_t, uint32_t) {
    const uint32_t pb = __shfl_up(b, 1, 64);
    const uint64_t ch = __ballot(lane == 0 || pb != b);
    if (b != HH_NOB && (lane == 0 || pb != b)) {
      const uint64_t rest = lane < 63 ? ch >> (lane + 1) : 0ull;
      atomicAdd(&s_h[b], rest ? (uint32_t)__builtin_ctzll(rest) + 1u : 64u - (uint32_t)lane);
    }
  };
  hh_enum_range(a, u, shift, h, fpr, f, j0, j1, s_incl, s_start, s_iv, s_w, &s_tot, count);
  if (!SCATTER) {
    for (uint32_t b = t; b < P; b += HH_NT)
      if (s_h[b]) atomicAdd(&bcnt[bb + b], s_h[b]);
    return;
  }
  __syncthreads();
  for (uint32_t b = t; b < P; b += HH_NT) {  // reserve: s_h[b] = this item's first scratch word in bucket b
    const uint32_t c = s_h[b];
    s_h[b] = c ? (uint32_t)boff[bb + b] + atomicAdd(&bcur[bb + b], c) : 0u;
  }
  __syncthreads();
  auto scatter = [&](uint32_t b, uint32_t w, uint32_t v) {
    const uint32_t pb = __shfl_up(b, 1, 64);
    const bool head = lane == 0 || pb != b;
    const uint64_t ch = __ballot(head);
    uint32_t base = 0;
    if (b != HH_NOB && head) {
      const uint64_t rest = lane < 63 ? ch >> (lane + 1) : 0ull;
      base = atomicAdd(&s_h[b], rest ? (uint32_t)__builtin_ctzll(rest) + 1u : 64u - (uint32_t)lane);
    }
    const uint64_t upto = ch & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
    const int hl = 63 - __builtin_clzll(upto);  // this lane's run head
    base = __shfl(base, hl, 64);
    if (b != HH_NOB) {
      const uint32_t p = base + (uint32_t)(lane - hl);
      sw[p] = w;
      if (CUSTOM) sv[p] = v;
    }
  };
  hh_enum_range(a, u, shift, h, fpr, f, j0, j1, s_incl, s_start, s_iv, s_w, &s_tot, scatter);
}

// Accumulation items {bucket, w-range [slo, shi), distinct bound}.  A bucket
// whose distinct-w bound 2 min(n, width) fits the table is one item
// (k_hh_plan).  A heavier one -- a hub row's wedges are skewed towards low
// ids, so its first buckets can hold most of them -- is cut into consecutive
// w-ranges from a histogram of its scratch: k_hh_plan lists the heavy buckets
// with their scratch in segments of HH_SEG wedges (one packed counter gives
// both the heavy index and the first segment, so segments stay sorted by
// heavy bucket), k_hh_hist histograms every segment over the bucket's bins
// (HH_BPS per segment, HH_FINE at most, power-of-two widths) in LDS and adds
// it to the bucket's global bins, and k_hh_group groups the bins greedily into
// ranges whose distinct-w bound min(wedges, width) stays within T / 2.  A
// single bin beyond that is one HH_WIDE item, accumulated in width sub-ranges
// of T / 2 by k_hh_accum.  The items of a heavy bucket run on different
// workgroups, each streaming the bucket's scratch and keeping its own w-range.
// Counts (every metric but AA / RA): a range no wider than dw (HH_DW) counts
// directly -- LDS counter [w - lo], one atomic add per wedge, no probing --
// when dense (wedges >= width / 4) or beyond the table's distinct bound; so a
// hub row's dense first buckets are single items.
// AA / RA sort mode (wcap = HH_SCAP): items hold at most HH_SCAP wedges, which
// k_hh_accum sorts by (w, v) in LDS and sums run by run in ascending v; a single
// bin beyond HH_SCAP wedges is flagged HH_BIG (hash table with the ordered
// re-walk of hp_ordered_sum).
struct HhItem {         // 64 bytes: everything k_hh_accum needs, one load
  uint32_t cnt;         // distinct-w bound of the range | HH_BIG | HH_WIDE | HH_DIRECT | HH_PART | HH_WHOLE
  uint32_t n;           // its wedges, at sw[off, off + n) (HH_PART: at pw)
  uint32_t u, du;       // the row and deg u
  uint64_t slo, shi;    // w-range
  uint64_t off;
  uint64_t x0, x1;      // the bucket's exclusion slice of N(u) (absolute entry indices)
  uint32_t gb, pad;     // bucket (statistics)
};
static_assert(sizeof(HhItem) == 64, "one 64-byte item");
constexpr uint32_t HH_FINE = 4096;
constexpr uint32_t HH_SCAP = 4096;         // sort-mode wedges per item (32 KB of u64 keys)
constexpr uint32_t HH_BIG = 0x80000000u;
constexpr uint32_t HH_WIDE = 0x40000000u;  // the range is accumulated in sub-ranges of cnt w
constexpr uint32_t HH_DIRECT = 0x20000000u;  // counts (no AA / RA) indexed by w - lo in LDS, no hashing
constexpr uint32_t HH_PART = 0x10000000u;    // a heavy bucket's item: its own wedges, partitioned by k_hh_part
constexpr uint32_t HH_WHOLE = 0x08000000u;   // every wedge at off is inside [slo, shi): no range test
constexpr uint32_t HH_CNT = 0x07ffffffu;
constexpr uint32_t HH_DW = 16384;          // direct counters per range (the two words of the 8192-entry table)
constexpr uint32_t HH_DMARK = 0x80000000u;  // direct counter: w is in N(u)
constexpr uint64_t HH_SEG = 65536;         // heavy scratch wedges per histogram segment
constexpr uint32_t HH_BPS = 512;           // histogram bins per segment
constexpr int HH_HSH = 40;                 // packed heavy counter: count << 40 | segments

struct HhHeavy {
  uint32_t gb, n;     // bucket, its wedges
  uint32_t nbin, fsh; // bins of width 2^fsh from lo
  uint64_t seg0;      // first segment (its bins at seg0 * HH_BPS)
  uint64_t lo, hi;    // the bucket's w-range
  uint32_t u, du;     // its row, deg u
  uint64_t x0, x1;    // its exclusion slice of N(u)
};

__device__ __forceinline__ uint64_t hh_bucket_range(const HpArgs& a, uint32_t u, uint32_t shift, uint64_t b,
                                                    uint64_t* lo) {
  *lo = (uint64_t)u + 1 + (b << shift);
  const uint64_t hi = *lo + (1ull << shift) < a.S ? *lo + (1ull << shift) : a.S;
  return hi - *lo;
}

// append with one atomic per wave (a single counter shared by the whole chip)
__device__ __forceinline__ uint32_t hh_wave_append(bool want, uint32_t* ctr) {
  const uint64_t m = __ballot(want);
  if (!m) return 0;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane_id() == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  return base + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1));
}

// The item word of a range of `span` w holding `cnt` wedges (counts mode, dw >
// 0 enables direct counting): 0 when neither the table nor direct counters fit.
__device__ __forceinline__ uint32_t hh_count_item(uint64_t cnt, uint64_t span, uint64_t th, uint32_t dw) {
  const uint64_t dist = cnt < span ? cnt : span;
  if (span <= dw && (dist > th || 4 * cnt >= span)) return (uint32_t)dist | HH_DIRECT;
  if (dist <= th) return (uint32_t)dist;
  return 0u;
}

// wcap > 0 (AA / RA sort mode, see k_hh_accum): items are bounded by their
// wedge count (<= wcap) instead of their distinct-w bound.  Heavy buckets go to
// heavy[] (at most hcap: host bound tot / half + 1) with their bins zeroed.
__global__ void k_hh_plan(HpArgs a, uint64_t nb, const uint32_t* __restrict__ brow, const uint32_t* __restrict__ hr_u,
                          const uint32_t* __restrict__ hr_shift, const uint32_t* __restrict__ hr_p,
                          const uint64_t* __restrict__ bbase, const uint64_t* __restrict__ boff,
                          const uint64_t* __restrict__ xs, const uint32_t* __restrict__ bcnt, int tl,
                          HhItem* __restrict__ items,
                          uint32_t* __restrict__ nitems, HhHeavy* __restrict__ heavy,
                          unsigned long long* __restrict__ hctr, uint64_t hcap, uint32_t* __restrict__ ghist,
                          uint32_t wcap, uint32_t dw) {
  const int lane = lane_id();
  const uint64_t th = 1ull << (tl - 1);
  for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < nb; b0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t gb = b0 + threadIdx.x;
    uint32_t n = 0, u = 0, du = 0;
    uint64_t lo = 0, width = 0, x0 = 0, x1 = 0;
    if (gb < nb) {
      n = bcnt[gb];
      const uint32_t r = brow[gb];
      u = hr_u[r];
      const uint64_t b = gb - bbase[r];
      width = hh_bucket_range(a, u, hr_shift[r], b, &lo);
      if (n) {
        const uint64_t o1 = a.g.off[u + 1];
        du = (uint32_t)(o1 - a.g.off[u]);
        x0 = xs[gb];
        x1 = b + 1 < hr_p[r] ? xs[gb + 1] : o1;  // N(u) entries in the bucket
      }
    }
    const uint64_t dist = (uint64_t)n < width ? (uint64_t)n : width;
    const uint32_t ci = wcap ? (n <= wcap ? (uint32_t)dist : 0u) : hh_count_item(n, width, th, dw);
    const bool simple = n > 0 && ci != 0, hv = n > 0 && !simple;
    const uint32_t i = hh_wave_append(simple, nitems);
    if (simple)  // i < nb <= the item capacity
      items[i] = HhItem{ci | HH_WHOLE, n, u, du, lo, lo + width, boff[gb], x0, x1, (uint32_t)gb, 0u};
    const uint64_t nseg = hv ? (n + HH_SEG - 1) / HH_SEG : 0;
    const uint64_t pk = hv ? (1ull << HH_HSH) | nseg : 0ull;
    const uint64_t inc = wave_incl_scan(pk), wt = __shfl(inc, 63, 64);
    unsigned long long base = 0;
    if (lane == 63 && wt) base = atomicAdd(hctr, (unsigned long long)wt);
    base = __shfl(base, 63, 64);
    if (hv) {
      const uint64_t ex = base + inc - pk;
      const uint64_t j = ex >> HH_HSH, s0 = ex & ((1ull << HH_HSH) - 1);
      const uint32_t nbin = (uint32_t)(nseg * HH_BPS < HH_FINE ? nseg * HH_BPS : HH_FINE);
      const uint32_t fsh = (uint32_t)log2_ceil((width + nbin - 1) / nbin);
      if (j < hcap) {
        heavy[j] = HhHeavy{(uint32_t)gb, n, nbin, fsh, s0, lo, lo + width, u, du, x0, x1};
        uint4* z = (uint4*)(ghist + s0 * HH_BPS);  // 16-byte aligned: HH_BPS words per segment
        for (uint32_t q = 0; q < nbin / 4; ++q) z[q] = make_uint4(0, 0, 0, 0);
      } else {
        atomicOr(&a.ctr[HPC_ERR], 4ull);
      }
    }
  }
}

// One workgroup per segment (grid-stride): its heavy bucket by binary search of
// the segments' starts, its wedges binned in LDS, the bins added to the bucket's.
__global__ __launch_bounds__(HH_NT) void k_hh_hist(HpArgs a, const HhHeavy* __restrict__ heavy,
                                                   const unsigned long long* __restrict__ hctr, uint64_t hcap,
                                                   const uint64_t* __restrict__ boff, const uint32_t* __restrict__ sw,
                                                   uint32_t* __restrict__ ghist) {
  __shared__ uint32_t s_h[HH_FINE];
  const int t = threadIdx.x, lane = lane_id();
  const uint64_t pk = *hctr;
  const uint64_t nh = (pk >> HH_HSH) < hcap ? (pk >> HH_HSH) : hcap, ns = pk & ((1ull << HH_HSH) - 1);
  for (uint64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    uint64_t lo = 0, hi = nh;  // the last heavy bucket with seg0 <= s (uniform: every thread the same loads)
    while (hi - lo > 1) {
      const uint64_t m = (lo + hi) >> 1;
      if (heavy[m].seg0 <= s) lo = m; else hi = m;
    }
    if (nh == 0) break;
    const HhHeavy hb = heavy[lo];
    const uint64_t i0 = (s - hb.seg0) * HH_SEG;
    if (i0 >= hb.n) continue;  // a segment of a bucket past hcap (HPC_ERR raised)
    const uint64_t i1 = i0 + HH_SEG < hb.n ? i0 + HH_SEG : hb.n;
    for (uint32_t f = t; f < hb.nbin; f += HH_NT) s_h[f] = 0;
    __syncthreads();
    const uint32_t* src = sw + boff[hb.gb];
    for (uint64_t j0 = i0; j0 < i1; j0 += (uint64_t)HH_NT * HP_UN) {
      uint32_t x[HP_UN];
#pragma unroll
      for (int q = 0; q < HP_UN; ++q) {
        const uint64_t j = j0 + (uint64_t)q * HH_NT + t;
        x[q] = src[j < i1 ? j : i0];
      }
#pragma unroll
      for (int q = 0; q < HP_UN; ++q) {
        // consecutive wedges of a sorted list fall in runs of equal bins: one LDS atomic per run
        const uint64_t j = j0 + (uint64_t)q * HH_NT + t;
        const uint32_t b = j < i1 ? (uint32_t)(((uint64_t)x[q] - hb.lo) >> hb.fsh) : HH_NOB;
        const uint32_t pb = __shfl_up(b, 1, 64);
        const bool head = lane == 0 || pb != b;
        const uint64_t ch = __ballot(head);
        if (b != HH_NOB && head) {
          const uint64_t rest = lane < 63 ? ch >> (lane + 1) : 0ull;
          atomicAdd(&s_h[b], rest ? (uint32_t)__builtin_ctzll(rest) + 1u : 64u - (uint32_t)lane);
        }
      }
    }
    __syncthreads();
    uint32_t* gh = ghist + hb.seg0 * HH_BPS;
    for (uint32_t f = t; f < hb.nbin; f += HH_NT)
      if (s_h[f]) atomicAdd(&gh[f], s_h[f]);
    __syncthreads();
  }
}

// One workgroup per heavy bucket (grid-stride): its bins into LDS, grouped
// greedily into the widest consecutive bin ranges that are one item each
// (wcap: at most wcap wedges; counts: hh_count_item).  The greedy walk is wave
// 0's, wave-uniform (a bin's count read from a register of 64 by readlane, the
// walk's state scalar); it records each group's bin range and count in LDS.
// Then the workgroup reserves the bucket's items contiguously, scans the
// counts (item g holds its wedges at [boff + pre_g, + cnt_g) of the
// partitioned scratch), writes the items, the cursors (HH_BPS words per
// segment past the bins, set to pre_g for k_hh_part) and overwrites each bin
// by its item.
__global__ __launch_bounds__(HH_NT) void k_hh_group(HpArgs a, const HhHeavy* __restrict__ heavy,
                                                    const unsigned long long* __restrict__ hctr, uint64_t hcap,
                                                    uint32_t* __restrict__ ghist, uint32_t* __restrict__ gcur,
                                                    const uint64_t* __restrict__ boff, int tl,
                                                    HhItem* __restrict__ items, uint32_t* __restrict__ nitems,
                                                    uint64_t cap, uint32_t wcap, uint32_t dw) {
  static_assert(HH_NT == NT, "block_excl_scan spans NT threads");
  constexpr int GPT = HH_FINE / HH_NT;  // groups per thread in the scan
  __shared__ uint32_t s_h[HH_FINE];
  __shared__ uint32_t s_gr[HH_FINE];    // group: first bin | end bin << 16
  __shared__ uint32_t s_gc[HH_FINE];    // group: wedges
  __shared__ uint64_t s_scan[NWAVE + 1];
  __shared__ uint32_t s_ng, s_base;
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t pk = *hctr;
  const uint64_t nh = (pk >> HH_HSH) < hcap ? (pk >> HH_HSH) : hcap;
  const uint64_t th = 1ull << (tl - 1);  // distinct w per table
  for (uint64_t hi = blockIdx.x; hi < nh; hi += gridDim.x) {
    const HhHeavy hb = heavy[hi];
    uint32_t* gh = ghist + hb.seg0 * HH_BPS;
    uint32_t* gc = gcur + hb.seg0 * HH_BPS;
    const uint32_t nbin = hb.nbin;
    for (uint32_t f = t; f < nbin; f += HH_NT) s_h[f] = gh[f];
    __syncthreads();
    // bins of width 2^fsh from lo cover the bucket, the last ones clipped to its end
    const uint64_t lo = hb.lo, end = hb.hi;
    auto rlo = [&](uint64_t f) { return lo + (f << hb.fsh) < end ? lo + (f << hb.fsh) : end; };
    auto item_word = [&](uint64_t f0, uint64_t f1, uint64_t cnt) {
      const uint64_t span = rlo(f1) - rlo(f0), dist = cnt < span ? cnt : span;
      if (wcap) {
        if (cnt <= wcap) return (uint32_t)dist;
        if (dist <= th) return (uint32_t)dist | HH_BIG;  // by hash, ordered re-walk
        return (uint32_t)th | HH_WIDE | HH_BIG;          // by width sub-ranges
      }
      const uint32_t c = hh_count_item(cnt, span, th, dw);
      return c ? c : (dw ? dw | HH_WIDE | HH_DIRECT : (uint32_t)th | HH_WIDE);
    };
    if (wv == 0) {
      // a range is fine as one item: sort mode by its wedges, counts by hh_count_item
      auto ok = [&](uint64_t f0, uint64_t f1, uint64_t cnt) {
        return cnt == 0 || (wcap ? cnt <= wcap : hh_count_item(cnt, rlo(f1) - rlo(f0), th, dw) != 0);
      };
      uint32_t ng = 0;
      auto group = [&](uint32_t f0, uint32_t f1, uint64_t cnt) {
        if (lane == 0) {
          s_gr[ng] = f0 | f1 << 16;
          s_gc[ng] = (uint32_t)cnt;
        }
        ++ng;
      };
      uint64_t acc = 0;
      uint32_t g0 = 0;
      for (uint32_t fb = 0; fb < nbin; fb += 64) {
        const uint32_t cv = fb + lane < nbin ? s_h[fb + lane] : 0u;
        const uint32_t lim = nbin - fb < 64 ? nbin - fb : 64;
        for (uint32_t q = 0; q < lim; ++q) {
          const uint32_t f = fb + q;
          const uint64_t c = (uint32_t)__builtin_amdgcn_readlane((int)cv, (int)q);
          if (!ok(f, f + 1, c)) {  // a bin beyond a group on its own
            if (acc) group(g0, f, acc);
            group(f, f + 1, c);
            acc = 0;
            g0 = f + 1;
          } else if (!ok(g0, f + 1, acc + c)) {
            group(g0, f, acc);
            acc = c;
            g0 = f;
          } else {
            if (!acc && !c) g0 = f + 1;
            acc += c;
          }
        }
      }
      if (acc) group(g0, nbin, acc);
      if (lane == 0) {
        s_ng = ng;
        s_base = atomicAdd(nitems, ng);
      }
    }
    __syncthreads();
    const uint32_t ng = s_ng, base = s_base;
    // pre_g: exclusive prefix of the group counts (GPT consecutive groups per thread)
    uint64_t mine = 0;
    for (int q = 0; q < GPT; ++q) {
      const uint32_t g = (uint32_t)t * GPT + q;
      if (g < ng) mine += s_gc[g];
    }
    uint64_t pre = block_excl_scan(mine, s_scan, nullptr);
    const uint64_t bo = boff[hb.gb];
    for (int q = 0; q < GPT; ++q) {
      const uint32_t g = (uint32_t)t * GPT + q;
      if (g >= ng) break;
      const uint32_t f0 = s_gr[g] & 0xffffu, f1 = s_gr[g] >> 16, cnt = s_gc[g];
      const uint64_t i = (uint64_t)base + g;
      if (i < cap)
        items[i] = HhItem{item_word(f0, f1, cnt) | HH_PART | HH_WHOLE, cnt, hb.u, hb.du, rlo(f0), rlo(f1), bo + pre,
                          hb.x0, hb.x1, hb.gb, 0u};
      else atomicOr(&a.ctr[HPC_ERR], 4ull);
      gc[g] = (uint32_t)pre;
      pre += cnt;
    }
    // bin -> its group: the last group starting at or before it (a bin before
    // every group, or between groups, is empty: no wedge maps there)
    for (uint32_t f = t; f < nbin; f += HH_NT) {
      uint32_t l = 0, h = ng;
      while (l < h) {
        const uint32_t m = (l + h) >> 1;
        if ((s_gr[m] & 0xffffu) <= f) l = m + 1; else h = m;
      }
      gh[f] = l ? l - 1 : HH_NOB;
    }
    __syncthreads();
  }
}

// The heavy buckets' wedges partitioned by item (one workgroup per segment,
// grid-stride): per item the segment's count in LDS, one global atomic per
// item reserves the segment's run of the item's range, a second read of the
// segment writes every wedge there (and v for AA / RA).  The order inside an
// item is free: its wedges are summed per w (counts), sorted (sort mode) or
// re-walked in N(u) order (HH_BIG).
__global__ __launch_bounds__(HH_NT) void k_hh_part(HpArgs a, const HhHeavy* __restrict__ heavy,
                                                   const unsigned long long* __restrict__ hctr, uint64_t hcap,
                                                   const uint64_t* __restrict__ boff, const uint32_t* __restrict__ sw,
                                                   const uint32_t* __restrict__ sv, const uint32_t* __restrict__ ghist,
                                                   uint32_t* __restrict__ gcur, uint32_t* __restrict__ pw,
                                                   uint32_t* __restrict__ pv) {
  __shared__ uint32_t s_map[HH_FINE];
  __shared__ uint32_t s_cnt[HH_FINE];
  const int t = threadIdx.x;
  const uint64_t pk = *hctr;
  const uint64_t nh = (pk >> HH_HSH) < hcap ? (pk >> HH_HSH) : hcap, ns = pk & ((1ull << HH_HSH) - 1);
  for (uint64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    uint64_t lo = 0, hi = nh;  // the last heavy bucket with seg0 <= s
    while (hi - lo > 1) {
      const uint64_t m = (lo + hi) >> 1;
      if (heavy[m].seg0 <= s) lo = m; else hi = m;
    }
    if (nh == 0) break;
    const HhHeavy hb = heavy[lo];
    const uint64_t i0 = (s - hb.seg0) * HH_SEG;
    if (i0 >= hb.n) continue;
    const uint64_t i1 = i0 + HH_SEG < hb.n ? i0 + HH_SEG : hb.n;
    const uint32_t* gm = ghist + hb.seg0 * HH_BPS;
    uint32_t* gc = gcur + hb.seg0 * HH_BPS;
    for (uint32_t f = t; f < hb.nbin; f += HH_NT) {
      s_map[f] = gm[f];
      s_cnt[f] = 0;
    }
    __syncthreads();
    const uint64_t bo = boff[hb.gb];
    const uint32_t* src = sw + bo;
    auto item_of = [&](uint32_t w) { return s_map[((uint64_t)w - hb.lo) >> hb.fsh]; };
    for (uint64_t j = i0 + t; j < i1; j += HH_NT) {
      const uint32_t g = item_of(src[j]);
      if (g < hb.nbin) atomicAdd(&s_cnt[g], 1u);
      else atomicOr(&a.ctr[HPC_ERR], 4ull);  // a wedge outside every item (never expected)
    }
    __syncthreads();
    for (uint32_t g = t; g < hb.nbin; g += HH_NT)  // items <= bins
      if (s_cnt[g]) s_cnt[g] = atomicAdd(&gc[g], s_cnt[g]);
    __syncthreads();
    for (uint64_t j = i0 + t; j < i1; j += HH_NT) {
      const uint32_t w = src[j], g = item_of(w);
      if (g >= hb.nbin) continue;
      const uint64_t p = bo + atomicAdd(&s_cnt[g], 1u);
      pw[p] = w;
      if (pv) pv[p] = sv[bo + j];
    }
    __syncthreads();
  }
}

// Ascending bitonic sort of n (a power of two, >= 2) u64 keys in LDS by the workgroup.
template <int NTH>
__device__ __forceinline__ void block_bitonic_u64(uint64_t* s, uint32_t n) {
  for (uint32_t k = 2; k <= n; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < n / 2; i += NTH) {
        const uint32_t lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
        const uint64_t x = s[lo], y = s[hi];
        if ((x > y) == ((lo & k) == 0)) {
          s[lo] = y;
          s[hi] = x;
        }
      }
      __syncthreads();
    }
}

// Sort-mode keys: (w - slo) << 38 | v << 12 | min(deg v, 4095) (w - slo, v < 2^26)
constexpr int HS_WSH = 38;
constexpr uint32_t HS_DMAX = 4095;
constexpr int HS_CT = 256;  // contributions cached in LDS by k_hh_accum's sort mode

// sortmode (AA / RA; nonzero: the plan's wedges per item, at most HH_SCAP, unless
// flagged HH_BIG -- those are cut into passes of at most that many): an
// item's wedges are loaded as (w, v, deg v) keys into LDS (over the vmin / vmax
// words of the hash table), sorted, and every run of equal w summed by its
// first thread in ascending v -- the additions of predict.hxx:788 / 828 in the
// reference's order; the exclusion marks the run of each x in N(u).
// TLC: log2 of the count metrics' table (the LDS it takes sets the workgroups
// per CU of this latency-bound kernel; k_hh_plan sizes the items for it)
template <bool CUSTOM, int TLC = HH_TL>
__global__ __launch_bounds__(HH_NT) void k_hh_accum(HpArgs a, const HhItem* __restrict__ items,
                                                    const uint32_t* __restrict__ nitems,
                                                    const uint32_t* __restrict__ sw0, const uint32_t* __restrict__ sv0,
                                                    const uint32_t* __restrict__ pw, const uint32_t* __restrict__ pv,
                                                    uint32_t* __restrict__ queue, int sortmode, uint64_t cap) {
  constexpr int TL = CUSTOM ? HH_TL - 1 : TLC;
  constexpr int LT = 1 << TL;
  constexpr int VT = CUSTOM ? LT : 1;
  static_assert(!CUSTOM || LT >= (int)HH_SCAP, "the sort buffer overlays the vmin / vmax words");
  __shared__ uint32_t s_tab[2 * LT];  // keys | counts; or direct counters (ranges of at most 2 LT w: the plan's dw)
  uint32_t* const s_k = s_tab;
  uint32_t* const s_c = s_tab + LT;
  __shared__ uint64_t s_vv[VT];  // vmin | vmax (2 x LT u32), or the sort-mode keys (LT u64)
  __shared__ uint8_t s_ex[CUSTOM ? HH_SCAP : 1];
  __shared__ uint32_t s_gu[HH_NW][HP_BSTG], s_gw[HH_NW][HP_BSTG];
  __shared__ float s_gs[HH_NW][HP_BSTG];
  __shared__ uint64_t s_item[8];  // the next item (8 words), loaded while this one runs
  __shared__ uint32_t s_tk[2];
  __shared__ uint32_t s_n;
  __shared__ uint32_t s_sp, s_rng[3];  // HH_BIG items: the range stack's size and the range being done,
  __shared__ uint32_t s_cur, s_grp[3];  // the next bin and the group cut from it
  __shared__ uint32_t s_w;              // the one w whose v-ranges are being added (thread 0: oacc)
  // AA / RA sort mode: the contributions c(d) of the degrees below HS_CT in
  // LDS -- every first hop of an LHub call up to H = 255 -- so a run's sum
  // waits on no global load (one dependent L2 round trip per run start was
  // the sort mode's critical path)
  __shared__ double s_ct[CUSTOM ? HS_CT : 1];
  const int t = threadIdx.x, wv = wave_id();
  if (CUSTOM)
    for (int i = t; i < HS_CT; i += HH_NT) s_ct[i] = (uint32_t)i < a.ctn ? a.g.ctab[i] : 0.0;
  uint32_t* const s_v0 = (uint32_t*)s_vv;
  uint32_t* const s_v1 = (uint32_t*)s_vv + (CUSTOM ? LT : 0);
  const HpTable tb{s_k, s_c, s_v0, s_v1};
  for (int i = t; i < LT; i += HH_NT) {
    s_k[i] = HP_EMPTY;
    s_c[i] = 0;
    if (CUSTOM) { s_v0[i] = HP_EMPTY; s_v1[i] = 0; }
  }
  HpStage sg{s_gu[wv], s_gw[wv], s_gs[wv], HP_BSTG, 0, 0, 0};
  const int64_t tau = *a.tau;
  // k_hh_group counts past `cap` when the item array overflows (and raises
  // HPC_ERR): never read beyond it
  const uint32_t ni = (uint32_t)min((uint64_t)*nitems, cap);
  uint64_t wedges = 0;
  float oacc = 0.0f;  // HH_BIG items, thread 0: the running sum of the one w (mode 2 - 4 below)
  // Items from the work queue two deep: while item `cur` runs, the next
  // ticket's item words and the ticket after it are in flight (a workgroup
  // barrier waits for LDS only, not for these loads), so an item costs no
  // queue or descriptor round trip of its own.
  if (t == 0) {
    s_tk[0] = atomicAdd(queue, 1u);
    s_tk[1] = atomicAdd(queue, 1u);
  }
  __syncthreads();
  uint32_t cur = s_tk[0], nx = s_tk[1];
  if (t < 8 && cur < ni) s_item[t] = ((const uint64_t*)(items + cur))[t];
  __syncthreads();
  // diagnostic (NLP_TRACE_HUB=1): the sort mode's phase times, thread 0's clock between barriers
  uint64_t ph_t = 0, ph_acc[5] = {0, 0, 0, 0, 0}, ph_max = 0;
  auto hh_mark = [&](int i) {
    if (a.ph && t == 0) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (i >= 0) ph_acc[i] += now - ph_t;
      if (i == 4 && now - ph_t > ph_max) ph_max = now - ph_t;
      ph_t = now;
    }
  };
  auto run = [&](const HhItem& item) {
    // a heavy bucket's item reads its own partitioned wedges
    const bool part = (item.cnt & HH_PART) != 0;
    const uint32_t* const sw = part ? pw : sw0;
    const uint32_t* const sv = part ? pv : sv0;
    const uint32_t n = item.n, u = item.u;
    const uint64_t off = item.off, du = item.du, x0 = item.x0, x1 = item.x1;
    const bool whole = (item.cnt & HH_WHOLE) != 0;
    const uint64_t slo = item.slo, shi = item.shi;
    if (CUSTOM && (item.cnt & HH_BIG) && t == 0) atomicAdd(&a.ctr[HPC_BIGW], (unsigned long long)n);
    // AA / RA sort mode: the wedges of [xlo, xhi) (at most HH_SCAP of them) as
    // (w, v, deg v) keys into LDS, sorted, every run of equal w summed by its
    // first thread in ascending v -- the reference's order of additions
    uint64_t* const sk = s_vv;
    auto sort_pass = [&](const uint64_t xlo, const uint64_t xhi, const bool all) {
        if (t == 0) s_n = 0;
        __syncthreads();
        hh_mark(-1);
        for (uint32_t i0 = 0; i0 < n; i0 += HH_NT * HP_UN) {
          uint32_t wq[HP_UN], vq[HP_UN], dq[HP_UN];
          bool in[HP_UN];
  #pragma unroll
          for (int k = 0; k < HP_UN; ++k) {
            const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
            const uint64_t p = off + (i < n ? i : 0u);
            wq[k] = sw[p];
            vq[k] = sv[p];
          }
  #pragma unroll
          for (int k = 0; k < HP_UN; ++k) {
            const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
            in[k] = i < n && (all || ((uint64_t)wq[k] >= xlo && (uint64_t)wq[k] < xhi));
            dq[k] = in[k] ? a.g.deg[vq[k]] : 0u;
          }
  #pragma unroll
          for (int k = 0; k < HP_UN; ++k) {
            const uint32_t pos = hh_wave_append(in[k], &s_n);  // one LDS atomic per wave
            if (in[k]) {
              ++wedges;
              if (pos < HH_SCAP)
                sk[pos] = ((uint64_t)wq[k] - xlo) << HS_WSH | (uint64_t)vq[k] << 12 |
                          (dq[k] < HS_DMAX ? dq[k] : HS_DMAX);
              else
                atomicOr(&a.ctr[HPC_ERR], 8ull);
            }
          }
        }
        __syncthreads();
        hh_mark(0);  // wedges loaded and appended
        const uint32_t m = s_n < HH_SCAP ? s_n : HH_SCAP;
        const uint32_t m2 = pow2_at_least(m);
        for (uint32_t i = m + t; i < m2; i += HH_NT) sk[i] = ~0ull;
        for (uint32_t i = t; i < m2; i += HH_NT) s_ex[i] = 0;
        __syncthreads();
        block_bitonic_u64<HH_NT>(sk, m2);
        hh_mark(1);  // sorted
        // first-order exclusion: the run of every x in N(u) within [xlo, xhi)
        hp_stream(a.g.keys + x0, x1 - x0, (uint32_t)t, (uint32_t)HH_NT, [&](uint32_t x) {
          if ((uint64_t)x >= xlo && (uint64_t)x < xhi) {
            const uint64_t xl = (uint64_t)x - xlo;
            uint32_t l = 0, h = m;
            while (l < h) {
              const uint32_t md = (l + h) >> 1;
              if ((sk[md] >> HS_WSH) < xl) l = md + 1; else h = md;
            }
            if (l < m && (sk[l] >> HS_WSH) == xl) s_ex[l] = 1;
          }
        });
        __syncthreads();
        hh_mark(2);  // exclusion marked
        for (uint32_t i0 = 0; i0 < m2; i0 += HH_NT) {
          const uint32_t i = i0 + (uint32_t)t;
          const bool start = i < m && (i == 0 || (sk[i] >> HS_WSH) != (sk[i - 1] >> HS_WSH));
          float s = 0.0f;
          uint32_t w = 0;
          if (start) {
            const uint64_t wl = sk[i] >> HS_WSH;
            float acc = 0.0f;
            for (uint32_t j = i; j < m && (sk[j] >> HS_WSH) == wl; ++j) {
              uint32_t d = (uint32_t)(sk[j] & 0xfffu);
              if (d == HS_DMAX) d = a.g.deg[(uint32_t)(sk[j] >> 12) & 0x3ffffffu];
              acc = (float)((double)acc + (d < (uint32_t)HS_CT ? s_ct[d] : a.g.ctab[d]));
            }
            s = s_ex[i] ? 0.0f : acc;
            w = (uint32_t)(xlo + wl);
          }
          hp_emit(sg, a, start, s, u, w, tau);
        }
        __syncthreads();
    };
    auto reset_vv = [&]() {  // the hash-table words under the sort buffer
      for (int i = t; i < LT; i += HH_NT) {
        s_v0[i] = HP_EMPTY;
        s_v1[i] = 0;
      }
      __syncthreads();
    };
    if (CUSTOM && sortmode && !(item.cnt & HH_BIG)) {
      hh_mark(-1);
      sort_pass(slo, shi, whole);
      hh_mark(3);  // runs summed, scored, emitted
      reset_vv();
      return;
    }
    if (CUSTOM && sortmode) {
      // an HH_BIG item (more than HH_SCAP wedges in one bin of the plan): cut
      // into w-ranges of at most `sortmode` wedges by histograms of its wedges
      // (ranges refined until they fit), each a sort pass; a single w with
      // more contributions than that is added over v-ranges in ascending v
      // (the reference's order: N(u) is sorted).  Round 5 took these items through the hash table
      // and re-walked N(u) x I(w) per entry with three or more contributions,
      // one thread each: one such item of C4 AA H = 32 took 840 ms.
      hh_mark(-1);
      uint32_t* const hist = s_k;   // LT bin counts
      // ranges to do: (lo, hi, mode) triples; mode 0 a w-range to cut, 2 one w,
      // 3 a v-range of that w, 4 that w's score
      uint32_t* const stk = s_c;
      constexpr uint32_t SCAP = LT / 3;
      if (t == 0) {
        stk[0] = (uint32_t)slo;
        stk[1] = (uint32_t)min(shi, (uint64_t)0xffffffffull);
        stk[2] = 0;
        s_sp = 1;
      }
      for (;;) {
        __syncthreads();
        if (s_sp == 0) break;
        if (t == 0) {
          const uint32_t q = --s_sp;
          s_rng[0] = stk[3 * q];
          s_rng[1] = stk[3 * q + 1];
          s_rng[2] = stk[3 * q + 2];
        }
        __syncthreads();
        const uint64_t lo = s_rng[0], hi = s_rng[1];
        const uint32_t mode = s_rng[2];
        if (mode == 2) {  // one w: its contributions over v-ranges (mode 3), then its score (mode 4)
          if (t == 0) {
            s_w = (uint32_t)lo;
            oacc = 0.0f;
            if (s_sp + 2 <= SCAP) {
              stk[3 * s_sp] = (uint32_t)lo;
              stk[3 * s_sp + 1] = (uint32_t)hi;
              stk[3 * s_sp + 2] = 4;
              stk[3 * s_sp + 3] = 0;
              stk[3 * s_sp + 4] = 1u << 26;  // sort mode: v < 2^26
              stk[3 * s_sp + 5] = 3;
              s_sp += 2;
            } else {
              atomicOr(&a.ctr[HPC_ERR], 16ull);
            }
          }
          continue;
        }
        if (mode == 4) {  // w's first-order exclusion (w in the item's slice of N(u): score 0) and emission
          bool ex = false;
          if (t == 0) {
            uint64_t l = x0, h = x1;
            while (l < h) {
              const uint64_t md = (l + h) >> 1;
              if ((uint64_t)a.g.keys[md] < lo) l = md + 1; else h = md;
            }
            ex = l < x1 && (uint64_t)a.g.keys[l] == lo;
          }
          hp_emit(sg, a, t == 0, ex ? 0.0f : oacc, u, (uint32_t)lo, tau);
          continue;
        }
        if (mode == 3) {
          // the one w's wedges with v in [lo, hi) in ascending v: a histogram of
          // their v over at most LT bins, groups of at most `sortmode` wedges
          // sorted and added by thread 0 in order; a bin beyond that is one v
          // (its equal contributions added in place) or refined: it and the rest
          // of the range go back onto the stack, the bin on top
          const uint32_t wv = s_w;
          int bsh = 0;
          while (((hi - lo + (1ull << bsh) - 1) >> bsh) > (uint64_t)LT) ++bsh;
          const uint32_t nb = (uint32_t)((hi - lo + (1ull << bsh) - 1) >> bsh);
          for (uint32_t i = t; i < nb; i += HH_NT) hist[i] = 0;
          __syncthreads();
          for (uint32_t i0 = 0; i0 < n; i0 += HH_NT * HP_UN) {
            uint32_t wq[HP_UN], vq[HP_UN];
#pragma unroll
            for (int k = 0; k < HP_UN; ++k) {
              const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
              const uint64_t p = off + (i < n ? i : 0u);
              wq[k] = sw[p];
              vq[k] = sv[p];
            }
#pragma unroll
            for (int k = 0; k < HP_UN; ++k) {
              const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
              if (i < n && wq[k] == wv && (uint64_t)vq[k] >= lo && (uint64_t)vq[k] < hi)
                atomicAdd(&hist[((uint64_t)vq[k] - lo) >> bsh], 1u);
            }
          }
          if (t == 0) s_cur = 0;
          for (;;) {
            __syncthreads();
            if (t == 0) {
              uint32_t c = s_cur;
              uint64_t acc = 0, g0 = lo + ((uint64_t)c << bsh);
              while (c < nb) {
                const uint32_t cnt = hist[c];
                const uint64_t b0 = lo + ((uint64_t)c << bsh), b1 = min(hi, b0 + (1ull << bsh));
                if (cnt > (uint32_t)sortmode) {
                  if (acc) break;
                  if (b1 - b0 == 1) {
                    const uint32_t d = a.g.deg[(uint32_t)b0];
                    const double cc = d < (uint32_t)HS_CT ? s_ct[d] : a.g.ctab[d];
                    for (uint32_t q = 0; q < cnt; ++q) oacc = (float)((double)oacc + cc);
                    wedges += cnt;
                    ++c;
                    g0 = b1;
                    continue;
                  }
                  if (s_sp + 2 <= SCAP) {
                    uint32_t q = s_sp;
                    if (b1 < hi) {
                      stk[3 * q] = (uint32_t)b1;
                      stk[3 * q + 1] = (uint32_t)hi;
                      stk[3 * q + 2] = 3;
                      ++q;
                    }
                    stk[3 * q] = (uint32_t)b0;
                    stk[3 * q + 1] = (uint32_t)b1;
                    stk[3 * q + 2] = 3;
                    s_sp = q + 1;
                  } else {
                    atomicOr(&a.ctr[HPC_ERR], 16ull);
                  }
                  c = nb;
                  break;
                }
                if (acc + cnt > (uint64_t)sortmode) break;
                acc += cnt;
                ++c;
              }
              s_cur = c;
              s_grp[0] = (uint32_t)g0;
              s_grp[1] = (uint32_t)(c < nb ? lo + ((uint64_t)c << bsh) : hi);
              s_grp[2] = acc ? 1u : 0u;
            }
            __syncthreads();
            if (!s_grp[2]) break;
            const uint32_t v0 = s_grp[0], v1 = s_grp[1];
            if (t == 0) s_n = 0;
            __syncthreads();
            for (uint32_t i0 = 0; i0 < n; i0 += HH_NT * HP_UN) {
              uint32_t wq[HP_UN], vq[HP_UN];
              bool in[HP_UN];
#pragma unroll
              for (int k = 0; k < HP_UN; ++k) {
                const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
                const uint64_t p = off + (i < n ? i : 0u);
                wq[k] = sw[p];
                vq[k] = sv[p];
              }
#pragma unroll
              for (int k = 0; k < HP_UN; ++k) {
                const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
                in[k] = i < n && wq[k] == wv && vq[k] >= v0 && vq[k] < v1;
                const uint32_t pos = hh_wave_append(in[k], &s_n);
                if (in[k]) {
                  ++wedges;
                  const uint32_t d = a.g.deg[vq[k]];
                  if (pos < HH_SCAP)
                    sk[pos] = (uint64_t)vq[k] << 12 | (d < HS_DMAX ? d : HS_DMAX);
                  else
                    atomicOr(&a.ctr[HPC_ERR], 8ull);
                }
              }
            }
            __syncthreads();
            const uint32_t m = s_n < HH_SCAP ? s_n : HH_SCAP;
            const uint32_t m2 = pow2_at_least(m);
            for (uint32_t i = m + t; i < m2; i += HH_NT) sk[i] = ~0ull;
            __syncthreads();
            block_bitonic_u64<HH_NT>(sk, m2);
            if (t == 0)
              for (uint32_t j = 0; j < m; ++j) {
                uint32_t d = (uint32_t)(sk[j] & 0xfffu);
                if (d == HS_DMAX) d = a.g.deg[(uint32_t)(sk[j] >> 12)];
                oacc = (float)((double)oacc + (d < (uint32_t)HS_CT ? s_ct[d] : a.g.ctab[d]));
              }
          }
          continue;
        }
        // mode 0: histogram [lo, hi) over at most LT bins, then group the bins
        int bsh = 0;
        while (((hi - lo + (1ull << bsh) - 1) >> bsh) > (uint64_t)LT) ++bsh;
        const uint32_t nb = (uint32_t)((hi - lo + (1ull << bsh) - 1) >> bsh);
        for (uint32_t i = t; i < nb; i += HH_NT) hist[i] = 0;
        __syncthreads();
        for (uint32_t i0 = 0; i0 < n; i0 += HH_NT * HP_UN) {
          uint32_t wq[HP_UN];
#pragma unroll
          for (int k = 0; k < HP_UN; ++k) {
            const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
            wq[k] = sw[off + (i < n ? i : 0u)];
          }
#pragma unroll
          for (int k = 0; k < HP_UN; ++k) {
            const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
            if (i < n && (uint64_t)wq[k] >= lo && (uint64_t)wq[k] < hi) atomicAdd(&hist[((uint64_t)wq[k] - lo) >> bsh], 1u);
          }
        }
        __syncthreads();
        // greedy groups of consecutive bins of at most `sortmode` (the plan's
        // capacity, HH_SCAP unless NLP_HASH_HUB_SCAP) wedges, each sorted
        // as soon as thread 0 has cut it (serial: rare items); a bin beyond that
        // goes onto the stack (refined, or one w)
        if (t == 0) s_cur = 0;
        for (;;) {
          __syncthreads();
          if (t == 0) {
            uint32_t c = s_cur;
            uint64_t acc = 0, g0 = lo + ((uint64_t)c << bsh);
            while (c < nb) {
              const uint32_t cnt = hist[c];
              const uint64_t b0 = lo + ((uint64_t)c << bsh), b1 = min(hi, b0 + (1ull << bsh));
              if (cnt > (uint32_t)sortmode) {
                if (acc) break;
                if (s_sp < SCAP) {
                  stk[3 * s_sp] = (uint32_t)b0;
                  stk[3 * s_sp + 1] = (uint32_t)b1;
                  stk[3 * s_sp + 2] = b1 - b0 == 1 ? 2u : 0u;
                  ++s_sp;
                } else {
                  atomicOr(&a.ctr[HPC_ERR], 16ull);  // more pending ranges than the stack holds: fail the call
                }
                ++c;
                g0 = b1;
                continue;
              }
              if (acc + cnt > (uint64_t)sortmode) break;
              acc += cnt;
              ++c;
            }
            s_cur = c;
            s_grp[0] = (uint32_t)g0;
            s_grp[1] = (uint32_t)(c < nb ? lo + ((uint64_t)c << bsh) : hi);
            s_grp[2] = acc ? 1u : 0u;
          }
          __syncthreads();
          if (!s_grp[2]) break;
          sort_pass(s_grp[0], s_grp[1], false);
        }
      }
      __syncthreads();
      for (int i = t; i < LT; i += HH_NT) {  // the hash table under the histogram and the stack
        s_k[i] = HP_EMPTY;
        s_c[i] = 0;
      }
      hh_mark(4);
      reset_vv();
      return;
    }
    if (!CUSTOM && (item.cnt & HH_DIRECT)) {
      // direct counters over sub-ranges of at most HH_DW w (HH_WIDE: of the item's count word)
      const uint64_t step = (item.cnt & HH_WIDE) ? (item.cnt & HH_CNT) : shi - slo;
      for (uint64_t xlo = slo; xlo < shi; xlo += step) {
        const uint64_t xhi = shi - xlo > step ? xlo + step : shi;
        const uint32_t span = (uint32_t)(xhi - xlo);
        const bool all = whole && step == shi - slo;
        if (span > 2u * LT) {  // a plan beyond the table (a sizing bug): fail the call, never overrun LDS
          if (t == 0) atomicOr(&a.ctr[HPC_ERR], 2ull);
          break;
        }
        for (uint32_t i = t; i < span; i += HH_NT) s_tab[i] = 0;
        __syncthreads();
        for (uint32_t i0 = 0; i0 < n; i0 += HH_NT * HH_AUN) {
          uint32_t wq[HH_AUN];
#pragma unroll
          for (int k = 0; k < HH_AUN; ++k) {
            const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
            wq[k] = sw[off + (i < n ? i : 0u)];
          }
#pragma unroll
          for (int k = 0; k < HH_AUN; ++k) {
            const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
            if (i < n && (all || ((uint64_t)wq[k] >= xlo && (uint64_t)wq[k] < xhi))) {
              ++wedges;
              atomicAdd(&s_tab[(uint64_t)wq[k] - xlo], 1u);
            }
          }
        }
        __syncthreads();
        // first-order exclusion: the entries of N(u) in [xlo, xhi) (a count stays: the entry is a candidate of count 0)
        hp_stream(a.g.keys + x0, x1 - x0, (uint32_t)t, (uint32_t)HH_NT, [&](uint32_t x) {
          if ((uint64_t)x >= xlo && (uint64_t)x < xhi) atomicOr(&s_tab[(uint64_t)x - xlo], HH_DMARK);
        });
        __syncthreads();
        for (uint32_t i0 = 0; i0 < span; i0 += HH_NT) {  // uniform trip count: hp_emit is wave-collective
          const uint32_t i = i0 + (uint32_t)t;
          uint32_t c = 0;
          if (i < span) {
            c = s_tab[i];
            s_tab[i] = i < (uint32_t)LT ? HP_EMPTY : 0u;  // the table's empty state again
          }
          const bool valid = (c & ~HH_DMARK) != 0;
          const uint32_t w = (uint32_t)(xlo + i);
          float sc = 0.0f;
          if (valid)
            sc = score_basic(a.metric, (c & HH_DMARK) ? 0u : c, du, a.metric != M_CN ? (uint64_t)a.g.deg[w] : 0ull);
          hp_emit(sg, a, valid, sc, u, w, tau);
        }
        __syncthreads();
      }
      return;
    }
    const uint32_t dcnt = item.cnt & HH_CNT;
    hh_mark(-1);
    const int lg = max(6, log2_ceil(2 * (uint64_t)dcnt));
    const uint32_t T = 1u << (lg < TL ? lg : TL), mask = T - 1;
    const int hs = 32 - (lg < TL ? lg : TL);
    // an HH_WIDE item: sub-ranges of dcnt w, each through the table
    const uint64_t step = (item.cnt & HH_WIDE) ? dcnt : shi - slo;
    // the first HH_XP x HH_NT keys of the exclusion slice are loaded with the
    // first wedges (one memory round trip fewer per item); the rest streams
    const uint64_t nx = x1 - x0;
    uint32_t xk[HH_XP];
#pragma unroll
    for (int q = 0; q < HH_XP; ++q) {
      const uint64_t i = (uint64_t)q * HH_NT + (uint64_t)t;
      xk[q] = i < nx ? a.g.keys[x0 + i] : 0u;
    }
    for (uint64_t xlo = slo; xlo < shi; xlo += step) {
      const uint64_t xhi = shi - xlo > step ? xlo + step : shi;
      const bool all = whole && step == shi - slo;
      for (uint32_t i0 = 0; i0 < n; i0 += HH_NT * HH_AUN) {
        uint32_t wq[HH_AUN], vq[HH_AUN];
#pragma unroll
        for (int k = 0; k < HH_AUN; ++k) {
          const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
          const uint64_t p = off + (i < n ? i : 0u);
          wq[k] = sw[p];
          vq[k] = CUSTOM ? sv[p] : 0u;
        }
#pragma unroll
        for (int k = 0; k < HH_AUN; ++k) {
          const uint32_t i = i0 + (uint32_t)k * HH_NT + (uint32_t)t;
          if (i < n && (all || ((uint64_t)wq[k] >= xlo && (uint64_t)wq[k] < xhi))) {
            ++wedges;
            hp_insert<false, CUSTOM>(tb, mask, hs, wq[k], vq[k], &a.ctr[HPC_ERR]);
          }
        }
      }
      __syncthreads();
      // first-order exclusion: the entries of N(u) in [xlo, xhi)
#pragma unroll
      for (int q = 0; q < HH_XP; ++q) {
        const uint32_t x = xk[q];
        if ((uint64_t)q * HH_NT + (uint64_t)t < nx && (uint64_t)x >= xlo && (uint64_t)x < xhi)
          hp_mark<false>(tb, mask, hs, x);
      }
      if (nx > (uint64_t)HH_XP * HH_NT)
        hp_stream(a.g.keys + x0 + (uint64_t)HH_XP * HH_NT, nx - (uint64_t)HH_XP * HH_NT, (uint32_t)t, (uint32_t)HH_NT,
                  [&](uint32_t x) {
                    if ((uint64_t)x >= xlo && (uint64_t)x < xhi) hp_mark<false>(tb, mask, hs, x);
                  });
      __syncthreads();
      hp_drain<false, CUSTOM, 8>(tb, T, (uint32_t)t, (uint32_t)HH_NT, sg, a, u, du, tau);
      __syncthreads();
    }
    hh_mark(4);  // a hash-table item (AA / RA: HH_BIG, with the ordered re-walk)
  };
  while (cur < ni) {
    HhItem item;
#pragma unroll
    for (int q = 0; q < 8; ++q) ((uint64_t*)&item)[q] = s_item[q];
    uint64_t pf = 0;
    uint32_t tk = 0;
    if (t < 8 && nx < ni) pf = ((const uint64_t*)(items + nx))[t];  // in flight during this item
    if (t == 0) tk = atomicAdd(queue, 1u);
    __syncthreads();  // every thread holds the item before s_item changes
    run(item);
    __syncthreads();
    if (t < 8) s_item[t] = pf;
    if (t == 0) s_tk[0] = tk;
    __syncthreads();
    cur = nx;
    nx = s_tk[0];
  }
  if (a.ph && t == 0) {
    for (int i = 0; i < 5; ++i) atomicAdd(&a.ph[i], (unsigned long long)ph_acc[i]);
    atomicMax(&a.ph[5], (unsigned long long)ph_max);  // the longest hash-table item
  }
  hp_finish(sg, a, wedges);
}

// ---------------------------------------------------------------- pruning between chunks
// Split the candidate buffer around the k-th key (sel[3] from the radix
// select): keys above go to the target columns (unordered), ties to a list of
// (u << 32 | w) records with their index, to be ordered canonically.
constexpr int HP_SPLIT_IPL = 16;  // elements per lane: a wave-tile = 1024 candidates, a workgroup tile 4 of them

// One pair of reservations (above, ties) per workgroup tile of 4096
// candidates: a chip-wide stream of atomics on two words serialises at their
// L2 channel, so the four waves' counts meet in LDS first.
__global__ __launch_bounds__(NT) void k_hp_split(const uint32_t* __restrict__ key, const uint32_t* __restrict__ u,
                                                 const uint32_t* __restrict__ w, const float* __restrict__ s, uint64_t n,
                                                 const uint64_t* __restrict__ sel, uint32_t* __restrict__ okey,
                                                 uint32_t* __restrict__ ou, uint32_t* __restrict__ ow,
                                                 float* __restrict__ os, uint64_t* __restrict__ tie_k,
                                                 uint32_t* __restrict__ tie_i, unsigned long long* __restrict__ cnt) {
  constexpr uint64_t WT = 64 * HP_SPLIT_IPL, BT = WT * NWAVE;
  __shared__ uint32_t s_na[NWAVE], s_nt[NWAVE];
  __shared__ unsigned long long s_base[2];
  const uint32_t kth = (uint32_t)sel[3];
  const int lane = lane_id(), wv = wave_id();
  const uint64_t below = (1ull << lane) - 1;
  const uint64_t nbt = (n + BT - 1) / BT;
  for (uint64_t bt = blockIdx.x; bt < nbt; bt += gridDim.x) {
    const uint64_t base = bt * BT + (uint64_t)wv * WT;
    uint32_t k[HP_SPLIT_IPL];
    uint32_t na = 0, nt = 0;
#pragma unroll
    for (int r = 0; r < HP_SPLIT_IPL; ++r) {
      const uint64_t i = base + (uint64_t)r * 64 + lane;
      k[r] = i < n ? key[i] : 0u;
      na += (uint32_t)__popcll(__ballot(i < n && k[r] > kth));
      nt += (uint32_t)__popcll(__ballot(i < n && k[r] == kth));
    }
    if (lane == 0) {
      s_na[wv] = na;
      s_nt[wv] = nt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t ta = 0, tt = 0;
      for (int q = 0; q < NWAVE; ++q) {
        ta += s_na[q];
        tt += s_nt[q];
      }
      s_base[0] = ta ? atomicAdd(&cnt[0], (unsigned long long)ta) : 0ull;
      s_base[1] = tt ? atomicAdd(&cnt[1], (unsigned long long)tt) : 0ull;
    }
    __syncthreads();
    unsigned long long pa = s_base[0], pt = s_base[1];
    for (int q = 0; q < wv; ++q) {
      pa += s_na[q];
      pt += s_nt[q];
    }
    __syncthreads();  // s_na / s_nt / s_base are rewritten by the next tile
#pragma unroll
    for (int r = 0; r < HP_SPLIT_IPL; ++r) {
      const uint64_t i = base + (uint64_t)r * 64 + lane;
      const bool above = i < n && k[r] > kth, tie = i < n && k[r] == kth;
      const uint64_t ma = __ballot(above), mt = __ballot(tie);
      if (above) {
        const uint64_t q = pa + __popcll(ma & below);
        okey[q] = k[r];
        ou[q] = u[i];
        ow[q] = w[i];
        os[q] = s[i];
      } else if (tie) {
        const uint64_t q = pt + __popcll(mt & below);
        tie_k[q] = ((uint64_t)u[i] << 32) | w[i];
        tie_i[q] = (uint32_t)i;
      }
      pa += __popcll(ma);
      pt += __popcll(mt);
    }
  }
}

// ---------------------------------------------------------------- tie selection (hp_prune)
// The first `quota` ties of the k-th key in (u, w) order, by a radix select
// over the packed keys (u << vb | w) -- four 13-bit digits from the top,
// ascending -- instead of sorting every tie: the kept set is all that the
// prune needs (the final order sorts it).  Needs 2 vb <= 52.
constexpr int TS_BITS = 13, TS_BINS = 1 << TS_BITS;
__device__ __forceinline__ uint64_t ts_key(uint64_t k, int vb) { return (k >> 32) << vb | (k & 0xffffffffull); }

// st: [0] prefix (the digits fixed so far), [1] remaining rank (1-based)
__global__ __launch_bounds__(NT) void k_ts_hist(const uint64_t* __restrict__ tk, uint64_t n, int vb, int shift,
                                                const uint64_t* __restrict__ st, uint32_t* __restrict__ ghist) {
  __shared__ uint32_t h[TS_BINS];
  for (int i = threadIdx.x; i < TS_BINS; i += NT) h[i] = 0;
  __syncthreads();
  const uint64_t prefix = st[0];
  const int ps = shift + TS_BITS;
  for (uint64_t j = (uint64_t)blockIdx.x * NT + threadIdx.x; j < n; j += (uint64_t)gridDim.x * NT) {
    const uint64_t k = ts_key(tk[j], vb);
    if ((k >> ps) == prefix) atomicAdd(&h[(k >> shift) & (TS_BINS - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TS_BINS; i += NT)
    if (h[i]) atomicAdd(&ghist[i], h[i]);
}

// One workgroup: the digit whose cumulative count (ascending) reaches the rank.
__global__ __launch_bounds__(NT) void k_ts_pick(uint32_t* __restrict__ ghist, uint64_t* __restrict__ st) {
  constexpr int PER = TS_BINS / NT;  // 32 bins per thread
  __shared__ uint64_t s_w[NWAVE];
  const int t = threadIdx.x;
  uint64_t mine = 0;
  for (int i = 0; i < PER; ++i) mine += ghist[t * PER + i];
  const uint64_t inc = wave_incl_scan(mine);
  if (lane_id() == 63) s_w[wave_id()] = inc;
  __syncthreads();
  uint64_t pre = 0;
  for (int q = 0; q < wave_id(); ++q) pre += s_w[q];
  const uint64_t excl = pre + inc - mine, rank = st[1];
  __syncthreads();
  if (excl < rank && rank <= excl + mine) {  // exactly one thread
    uint64_t rem = rank - excl;
    int d = t * PER;
    for (; d < t * PER + PER - 1; ++d) {
      const uint64_t c = ghist[d];
      if (c >= rem) break;
      rem -= c;
    }
    st[0] = (st[0] << TS_BITS) | (uint64_t)d;
    st[1] = rem;
  }
  __syncthreads();
  for (int i = t; i < TS_BINS; i += NT) ghist[i] = 0;  // ready for the next pass
}

// The ties with packed key <= st[0] (exactly the quota: keys are unique)
// behind the `above` entries, in any order; one reservation per workgroup tile.
__global__ __launch_bounds__(NT) void k_ts_take(const uint64_t* __restrict__ tk, const uint32_t* __restrict__ ti,
                                                uint64_t n, int vb, const uint64_t* __restrict__ st, uint64_t above,
                                                const uint32_t* __restrict__ key, const uint32_t* __restrict__ u,
                                                const uint32_t* __restrict__ w, const float* __restrict__ s,
                                                uint32_t* __restrict__ okey, uint32_t* __restrict__ ou,
                                                uint32_t* __restrict__ ow, float* __restrict__ os,
                                                unsigned long long* __restrict__ cnt) {
  constexpr int IPL = 8;
  constexpr uint64_t WT = 64 * IPL, BT = WT * NWAVE;
  __shared__ uint32_t s_n[NWAVE];
  __shared__ unsigned long long s_base;
  const uint64_t thr = st[0];
  const int lane = lane_id(), wv = wave_id();
  const uint64_t below = (1ull << lane) - 1;
  const uint64_t nbt = (n + BT - 1) / BT;
  for (uint64_t bt = blockIdx.x; bt < nbt; bt += gridDim.x) {
    const uint64_t base = bt * BT + (uint64_t)wv * WT;
    bool sel[IPL];
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < IPL; ++r) {
      const uint64_t j = base + (uint64_t)r * 64 + lane;
      sel[r] = j < n && ts_key(tk[j], vb) <= thr;
      c += (uint32_t)__popcll(__ballot(sel[r]));
    }
    if (lane == 0) s_n[wv] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (int q = 0; q < NWAVE; ++q) tot += s_n[q];
      s_base = tot ? atomicAdd(cnt, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    unsigned long long p = s_base;
    for (int q = 0; q < wv; ++q) p += s_n[q];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < IPL; ++r) {
      const uint64_t m = __ballot(sel[r]);
      if (sel[r]) {
        const uint64_t q = above + p + __popcll(m & below);
        const uint32_t i = ti[base + (uint64_t)r * 64 + lane];
        okey[q] = key[i];
        ou[q] = u[i];
        ow[q] = w[i];
        os[q] = s[i];
      }
      p += __popcll(m);
    }
  }
}

// the first `take` ties (canonical order) behind the `above` entries
__global__ void k_hp_take(const uint32_t* __restrict__ idx, uint64_t take, uint64_t above,
                          const uint32_t* __restrict__ key, const uint32_t* __restrict__ u,
                          const uint32_t* __restrict__ w, const float* __restrict__ s, uint32_t* __restrict__ okey,
                          uint32_t* __restrict__ ou, uint32_t* __restrict__ ow, float* __restrict__ os) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < take; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = idx[j];
    okey[above + j] = key[i];
    ou[above + j] = u[i];
    ow[above + j] = w[i];
    os[above + j] = s[i];
  }
}

__device__ __forceinline__ float score_of_key(uint32_t key) {
  return __uint_as_float((key & 0x80000000u) ? (key & 0x7fffffffu) : ~key);
}


}  // namespace nlp
