// group.hpp -- wedge generation into per-source buckets and per-bucket grouping.
//
// A wedge (u, v, w) is stored in u's bucket as the 64-bit record (w << 32 | v).
// Sorting a bucket by record value groups equal w together AND orders each
// group by v ascending, which is exactly the order in which the reference adds
// the contributions of v to entry w of u's counter table (v walks the sorted
// list N(u), predict.hxx:298-304; duplicates of v are consecutive and add the
// same value).  So the count (basic metrics) and the float accumulation
// (Adamic-Adar / Resource-Allocation, predict.hxx:788, 828) are reproduced
// bit-exactly without any global sort.
//
// Buckets of <= 32 records are sorted in registers by a bitonic network with
// compile-time indices (one thread per source vertex); larger ones go to a
// work list processed one workgroup per bucket with an LDS bitonic sort
// (<= BIG_CAP records; beyond that the host falls back to the radix path).
#pragma once
#include "kernels.hpp"
#include "lookback.hpp"

namespace nlp {

constexpr uint32_t SMALL_MAX = 16;   // buckets sorted in registers by one thread
constexpr uint32_t WAVE_MAX = 512;   // buckets sorted in LDS by one wave
constexpr uint32_t BIG_CAP = 8192;   // buckets sorted in LDS by one workgroup (64 KiB)
constexpr int GT_IPT = 4;
constexpr int GT_TILE = NT * GT_IPT; // sources per workgroup tile

// Per-call device counters (zeroed with the arena).
enum {
  C_NV = 0,      // surviving intermediates
  C_E = 1,       // in-edges of surviving intermediates (path 1) / edges (path 2)
  C_W = 2,       // wedges in buckets
  C_C = 3,       // candidates after compaction
  C_NBIG = 4,    // buckets on the big list
  C_NAN = 5,     // NaN candidates
  C_FLAGS = 6,   // bit 0: capacity overflow, bit 1: bucket > BIG_CAP, bit 2+: look-back timeout
  C_N_URANGE = 7,// ub - ua (scan length of the bucket scan)
  C_CBASE = 8,   // candidates already in the output buffer (path 2 chunks)
  C_WBASE = 9,   // first wedge slot of this chunk (path 2)
  NCTR = 16
};
constexpr uint64_t F_OVERFLOW = 1, F_TOOBIG = 2;
// the counted ordering passes (k_sp_cpass) got more than CP_MAXT tiles: the call is redone with look-back passes
constexpr uint64_t F_CPASS = 4;
constexpr uint64_t F_SMALL = 8;  // k_sp_order_rank: more candidates than SO_MAX (redo with the counted passes)

struct GraphView {
  const uint64_t* off;
  const uint32_t* keys;
  const uint32_t* deg;
  const uint64_t* toff;
  const uint32_t* tkeys;
  const double* ctab;
  const uint32_t* efilt;  // edge filter: bit edge_slot(u, w) set for every adjacency entry w in N(u)
  uint32_t efbits;        // log2 of its bit count (0: no filter)
  uint32_t maxf2;         // MAXFACTOR2 (0: off)
  const uint64_t* etab;   // exact membership table of the entries (u, w), w > u (null: none)
  uint32_t etbits;        // log2 of its bucket count
};

// The reference's MAXFACTOR2 filter on second-hop keys (predict.hxx:221,295):
// ft(w) = w > u && deg(u) <= F deg(u) && deg(w) <= F deg(u), size_t products.
// Its first clause holds for F >= 1; the second is a per-(u, w) predicate, so a
// w it rejects is never counted, never touched and never a candidate -- the
// same as dropping the pair where it is scored.
__device__ __forceinline__ bool f2_drop(const GraphView& g, uint32_t u, uint32_t w) {
  return g.maxf2 != 0 && (uint64_t)g.deg[w] > (uint64_t)g.maxf2 * (uint64_t)g.deg[u];
}

// Slot of (u, w) in the edge filter: a 64-bit mix (murmur3 finaliser), top bits.
__device__ __forceinline__ uint64_t edge_slot(uint32_t u, uint32_t w, uint32_t bits) {
  uint64_t x = ((uint64_t)u << 32) | w;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x >> (64 - bits);
}

// w in N(u)?  (u < w; the table when there is one -- behind the edge filter
// when both exist (NLP_EDGE_FILTER=2): a clear bit proves absence -- else a
// search of N(u))
__device__ __forceinline__ bool first_order(const GraphView& g, uint32_t u, uint32_t w) {
  if (g.etab) {
    if (g.efbits) {
      const uint64_t h = edge_slot(u, w, g.efbits);
      if (!((g.efilt[h >> 5] >> (h & 31)) & 1u)) return false;
    }
    return et_has(g.etab, g.etbits, u, w);
  }
  return contains_u32(g.keys + g.off[u], g.deg[u], w);
}

// One wave per row u: set the filter bit of every (u, w), w in N(u).
__global__ __launch_bounds__(256) void k_edge_filter(const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                                                     uint64_t S, uint32_t* __restrict__ filt, uint32_t bits) {
  const uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= S) return;
  const uint64_t a = off[u], b = off[u + 1];
  for (uint64_t j = a + (threadIdx.x & 63); j < b; j += 64) {
    const uint64_t h = edge_slot((uint32_t)u, keys[j], bits);
    atomicOr(&filt[h >> 5], 1u << (h & 31));
  }
}

// ---------------------------------------------------------------- path 1 scans
// Compaction of surviving intermediates v (0 < deg v <= H, |I(v)| > 0); also
// zeroes the bucket counters of the source range (same index space).
struct F_VSelect {
  const uint32_t* deg;
  const uint64_t* toff;
  uint32_t H;
  uint64_t ua, ub;
  uint32_t* ucnt;
  uint32_t* vlist;
  uint8_t* cache;  // pass A's flags, so pass B reads 1 byte per vertex
  __device__ uint64_t count(uint64_t v) const {
    if (v >= ua && v < ub) ucnt[v] = 0;
    uint32_t d = deg[v];
    return (d > 0 && d <= H && toff[v + 1] > toff[v]) ? 1 : 0;
  }
  __device__ uint64_t count_a(uint64_t v) const {
    uint64_t c = count(v);
    cache[v] = (uint8_t)c;
    return c;
  }
  __device__ uint64_t count_b(uint64_t v) const { return cache[v]; }
  __device__ void emit(uint64_t v, uint64_t off, uint64_t c) const {
    if (c) vlist[off] = (uint32_t)v;
  }
};

// In-edge offsets of the surviving intermediates.
struct F_VInOff {
  const uint32_t* vlist;
  const uint64_t* toff;
  uint64_t* vioff;
  __device__ uint64_t count(uint64_t j) const {
    uint32_t v = vlist[j];
    return toff[v + 1] - toff[v];
  }
  __device__ uint64_t count_a(uint64_t j) const { return count(j); }
  __device__ uint64_t count_b(uint64_t j) const { return count(j); }
  __device__ void emit(uint64_t j, uint64_t off, uint64_t) const { vioff[j] = off; }
};

// Bucket offsets over the source range (relative to ua).
struct F_UOff {
  const uint32_t* ucnt;
  uint64_t* uoff;
  uint64_t ua;
  __device__ uint64_t count(uint64_t i) const { return ucnt[ua + i]; }
  __device__ uint64_t count_a(uint64_t i) const { return count(i); }
  __device__ uint64_t count_b(uint64_t i) const { return count(i); }
  __device__ void emit(uint64_t i, uint64_t off, uint64_t) const { uoff[ua + i] = off; }
};

// One thread per in-edge slot e (v from the compact list): reserve the wedge
// slots of (v -> u) in u's bucket.  ie_u = u, ie_v = v, ie_first = index in N(v)
// of the first w > u (== deg v when there is none), ie_pos = offset in u's bucket.
__global__ void k_p1_reserve(GraphView g, const uint32_t* __restrict__ vlist, const uint64_t* __restrict__ vioff,
                             const uint64_t* __restrict__ ctr, uint64_t capE, uint64_t ua, uint64_t ub,
                             uint32_t* __restrict__ ucnt, uint32_t* __restrict__ ie_u, uint32_t* __restrict__ ie_v,
                             uint32_t* __restrict__ ie_first, uint32_t* __restrict__ ie_pos,
                             uint64_t* __restrict__ flags) {
  const uint64_t E = ctr[C_E], nV = ctr[C_NV];
  if (E > capE) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long*)flags, F_OVERFLOW);
    return;
  }
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t jv = lbs_find(vioff, nV, e);
    uint32_t v = vlist[jv];
    uint32_t u = g.tkeys[g.toff[v] + (e - vioff[jv])];
    uint32_t d = g.deg[v];
    uint32_t first = d;
    uint32_t pos = 0;
    if (u >= ua && u < ub) {
      first = upper_bound_u32(g.keys + g.off[v], d, u);
      if (first < d) pos = atomicAdd(&ucnt[u], d - first);
    }
    ie_u[e] = u;
    ie_v[e] = v;
    ie_first[e] = first;
    ie_pos[e] = pos;
  }
}

// Fill the reserved bucket slots with (w << 32 | v).
__global__ void k_p1_fill(GraphView g, const uint64_t* __restrict__ ctr, uint64_t capE, uint64_t capW,
                          const uint64_t* __restrict__ uoff, const uint32_t* __restrict__ ie_u,
                          const uint32_t* __restrict__ ie_v, const uint32_t* __restrict__ ie_first,
                          const uint32_t* __restrict__ ie_pos, uint64_t* __restrict__ bucket,
                          uint64_t* __restrict__ flags) {
  const uint64_t E = ctr[C_E], W = ctr[C_W];
  if (E > capE) return;
  if (W > capW) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long*)flags, F_OVERFLOW);
    return;
  }
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t v = ie_v[e], first = ie_first[e];
    uint32_t d = g.deg[v];
    if (first >= d) continue;
    uint64_t b = uoff[ie_u[e]] + ie_pos[e];
    const uint32_t* nv = g.keys + g.off[v];
    for (uint32_t i = first; i < d; ++i) bucket[b + (i - first)] = ((uint64_t)nv[i] << 32) | v;
  }
}

// ---------------------------------------------------------------- path 1, streaming form
// Two passes over all vertices v (no list of survivors: appending to one
// global counter would serialise tens of thousands of atomics on one word).
// A survivor is 0 < deg v <= H; for each in-neighbour u (transposed list I(v))
// inside the source range, the wedges (u, v, w) with w > u, w in N(v).
// Pass 1 adds the counts to ucnt[u]; pass 2 writes the records into u's
// bucket at slots drawn from cursor[u] (their order inside a bucket is
// irrelevant: buckets are sorted by record).  ucnt and cursor are all-zero on
// entry: k_group_tiles zeroes what it reads.
constexpr int P1_IPT = 8;
constexpr int P1_TILE = NT * P1_IPT;  // vertices per workgroup iteration
constexpr int P1_Q = 1024;             // queued (v, in-edge) pairs (16 KiB of LDS)

// Per (v, in-edge j) pair: the wedges (u = I(v)[j], v, w > u).
template <bool FILL>
__device__ __forceinline__ void p1_pair(const GraphView& g, uint32_t v, uint32_t d, uint64_t j, uint64_t ua,
                                        uint64_t ub, uint32_t* __restrict__ cnt, const uint64_t* __restrict__ uoff,
                                        uint64_t* __restrict__ bucket) {
  const uint32_t u = g.tkeys[j];
  if (u < ua || u >= ub) return;
  const uint32_t* nv = g.keys + g.off[v];
  const uint32_t first = upper_bound_u32(nv, d, u);
  if (first >= d) return;
  if (!FILL) {
    atomicAdd(&cnt[u], d - first);
  } else {
    const uint64_t b = uoff[u] + atomicAdd(&cnt[u], d - first);
    for (uint32_t k = first; k < d; ++k) bucket[b + (k - first)] = ((uint64_t)nv[k] << 32) | v;
  }
}

// Each workgroup scans P1_TILE vertices with independent coalesced loads,
// queues the (v, in-edge) pairs of the survivors in LDS, then processes one
// pair per thread, so that the dependent chains of different pairs overlap.
template <bool FILL>
__global__ __launch_bounds__(NT) void k_p1_pass(GraphView g, uint64_t S, uint32_t H, uint64_t ua, uint64_t ub,
                                                uint32_t* __restrict__ cnt, const uint64_t* __restrict__ uoff,
                                                uint64_t capW, uint64_t* __restrict__ bucket,
                                                uint64_t* __restrict__ ctr) {
  __shared__ uint32_t q_v[P1_Q];
  __shared__ uint32_t q_d[P1_Q];
  __shared__ uint64_t q_j[P1_Q];
  __shared__ uint32_t n_q;
  if (FILL && ctr[C_W] > capW) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_OVERFLOW);
    return;
  }
  for (uint64_t t0 = (uint64_t)blockIdx.x * P1_TILE; t0 < S; t0 += (uint64_t)gridDim.x * P1_TILE) {
    if (threadIdx.x == 0) n_q = 0;
    __syncthreads();
    uint32_t dd[P1_IPT];
#pragma unroll
    for (int i = 0; i < P1_IPT; ++i) {
      const uint64_t v = t0 + (uint64_t)i * NT + threadIdx.x;
      dd[i] = v < S ? g.deg[v] : 0u;
    }
#pragma unroll
    for (int i = 0; i < P1_IPT; ++i) {
      const uint64_t v = t0 + (uint64_t)i * NT + threadIdx.x;
      const uint32_t d = dd[i];
      if (d == 0 || d > H) continue;
      const uint64_t a = g.toff[v], b = g.toff[v + 1];
      if (b == a) continue;
      const uint32_t r = (uint32_t)std::min<uint64_t>(b - a, P1_Q);
      const uint32_t k = atomicAdd(&n_q, r);
      if (k + (b - a) <= P1_Q) {
        for (uint64_t j = a; j < b; ++j) {
          q_v[k + (j - a)] = (uint32_t)v;
          q_d[k + (j - a)] = d;
          q_j[k + (j - a)] = j;
        }
      } else {  // queue full (large in-degree): this thread handles its pairs itself
        for (uint32_t x = k; x < P1_Q && x < k + r; ++x) q_d[x] = 0;  // reserved slots stay empty
        for (uint64_t j = a; j < b; ++j) p1_pair<FILL>(g, (uint32_t)v, d, j, ua, ub, cnt, uoff, bucket);
      }
    }
    __syncthreads();
    const uint32_t nq = std::min<uint32_t>(n_q, P1_Q);
    for (uint32_t q = threadIdx.x; q < nq; q += NT) {
      if (q_d[q] == 0) continue;
      p1_pair<FILL>(g, q_v[q], q_d[q], q_j[q], ua, ub, cnt, uoff, bucket);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- path 2 (source-centric) scans
// Per edge e of the source range [e0, e0+n): wedges (u, v, w>u) through v if v
// survives the hub filter (predict.hxx:301).
struct F_EdgeWc {
  GraphView g;
  uint64_t span, e0;
  uint32_t H;
  uint64_t* woff;
  __device__ uint64_t count(uint64_t i) const {
    uint64_t e = e0 + i;
    uint32_t v = g.keys[e];
    uint32_t d = g.deg[v];
    if (H != 0 && d > H) return 0;
    uint32_t u = (uint32_t)lbs_find(g.off, span + 1, e);
    return d - upper_bound_u32(g.keys + g.off[v], d, u);
  }
  __device__ void emit(uint64_t i, uint64_t off, uint64_t) const { woff[i] = off; }
};

// Fill the wedge slots of edges [a, b) (relative), chunk starting at slot wa.
__global__ void k_p2_fill(GraphView g, uint64_t span, uint64_t e0, uint64_t a, uint64_t b, uint64_t wa, uint32_t H,
                          const uint64_t* __restrict__ woff, uint64_t* __restrict__ bucket) {
  for (uint64_t i = a + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t e = e0 + i;
    uint32_t v = g.keys[e];
    uint32_t d = g.deg[v];
    if (H != 0 && d > H) continue;
    uint64_t s = woff[i], t = woff[i + 1];
    if (s == t) continue;
    uint32_t first = d - (uint32_t)(t - s);
    const uint32_t* nv = g.keys + g.off[v];
    for (uint64_t j = 0; j < t - s; ++j) bucket[s - wa + j] = ((uint64_t)nv[first + j] << 32) | v;
  }
}

// ---------------------------------------------------------------- bucket views
struct BucketsP1 {  // per source u: [uoff[u], uoff[u] + ucnt[u])
  const uint64_t* uoff;
  const uint32_t* ucnt;
  __device__ void get(uint64_t u, uint64_t& s, uint32_t& c) const {
    c = ucnt[u];
    s = c ? uoff[u] : 0;
  }
};
struct BucketsP2 {  // per source u of the chunk: from the per-edge wedge offsets
  const uint64_t* off;
  const uint64_t* woff;
  uint64_t e0, wa;
  __device__ void get(uint64_t u, uint64_t& s, uint32_t& c) const {
    uint64_t a = woff[off[u] - e0], b = woff[off[u + 1] - e0];
    s = a - wa;
    c = (uint32_t)(b - a);
  }
};

// ---------------------------------------------------------------- scoring of one (u, w) run
struct Stage {  // candidate staging, indexed by bucket slot
  uint32_t* key;
  uint32_t* u;
  uint32_t* w;
  float* s;
  uint32_t* flag;
};

// Record one (u, w) run in the staging slot of its first wedge; scoring happens
// in k_score_runs, one thread per run, so that the membership searches of
// different runs proceed in parallel instead of back to back in one thread.
template <bool CUSTOM>
__device__ __forceinline__ void emit_run(const GraphView&, int, float, uint32_t u, uint32_t w, uint32_t count,
                                         float acc, uint64_t slot, const Stage& st) {
  st.u[slot] = u;
  st.w[slot] = w;
  if (CUSTOM) st.s[slot] = acc;
  else st.key[slot] = count;
  st.flag[slot] = 1u;
}

// One thread per staging slot: first-order exclusion (predict.hxx:306-307),
// the metric's score (fs), the score <= minScore filter (predict.hxx:311).
template <bool CUSTOM>
__global__ __launch_bounds__(NT) void k_score_runs(GraphView g, int metric, float min_score,
                                                   const uint64_t* __restrict__ ctr, uint64_t capW, Stage st) {
  const uint64_t W = ctr[C_W];
  if (W > capW || (ctr[C_FLAGS] & F_OVERFLOW)) return;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < W; i += (uint64_t)gridDim.x * blockDim.x) {
    if (!st.flag[i]) continue;
    const uint32_t u = st.u[i], w = st.w[i];
    const bool excl = first_order(g, u, w);
    float sc;
    if (CUSTOM) sc = excl ? 0.0f : st.s[i];
    else sc = score_basic(metric, excl ? 0u : st.key[i], g.deg[u], g.deg[w]);
    st.key[i] = score_key(sc);
    st.s[i] = sc;
    st.flag[i] = (!(sc <= min_score) && !f2_drop(g, u, w)) ? 1u : 0u;  // NaN passes
  }
}

template <int N>
__device__ __forceinline__ void bitonic_regs(uint64_t (&a)[N]) {
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          uint64_t x = a[i], y = a[l];
          bool sw = up ? (x > y) : (x < y);
          a[i] = sw ? y : x;
          a[l] = sw ? x : y;
        }
      }
    }
  }
}

template <int N, bool CUSTOM>
__device__ __forceinline__ void group_small(const GraphView& g, int metric, float min_score, uint32_t u,
                                            const uint64_t* __restrict__ bucket, uint64_t s, uint32_t c,
                                            const Stage& st) {
  uint64_t a[N];
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = (uint32_t)i < c ? bucket[s + i] : ~0ull;
  bitonic_regs<N>(a);
  uint32_t cur = (uint32_t)(a[0] >> 32), rs = 0, cnt = 0;
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if ((uint32_t)i < c) {
      uint32_t w = (uint32_t)(a[i] >> 32);
      if (i > 0 && w != cur) {
        emit_run<CUSTOM>(g, metric, min_score, u, cur, cnt, acc, s + rs, st);
        cur = w;
        rs = i;
        cnt = 0;
        acc = 0.0f;
      }
      ++cnt;
      if (CUSTOM) acc = (float)((double)acc + g.ctab[g.deg[(uint32_t)a[i]]]);
      if ((uint32_t)i != rs) st.flag[s + i] = 0u;
    }
  }
  emit_run<CUSTOM>(g, metric, min_score, u, cur, cnt, acc, s + rs, st);
}

// LDS ordering point for one wave: every lane's LDS writes before, reads after.
// Workgroup-scope fences: a wavefront-scope fence emits no instruction and the
// scheduler may move DS accesses across it (path 4).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Sort r[0..c) (padded to a power of two >= 64) in LDS by one wave, then walk
// the runs: lane i owns the runs that start at its strided slots.
template <bool CUSTOM>
__device__ __forceinline__ void group_wave(const GraphView& g, int metric, float min_score, uint32_t u,
                                           const uint64_t* __restrict__ bucket, uint64_t s, uint32_t c,
                                           uint64_t* r, const Stage& st) {
  const int lane = lane_id();
  uint32_t n2 = 64;
  while (n2 < c) n2 <<= 1;
  for (uint32_t i = lane; i < n2; i += 64) r[i] = i < c ? bucket[s + i] : ~0ull;
  wave_lds_sync();
  for (uint32_t k = 2; k <= n2; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = lane; i < n2; i += 64) {
        uint32_t l = i ^ j;
        if (l > i) {
          bool up = (i & k) == 0;
          uint64_t x = r[i], y = r[l];
          if (up ? (x > y) : (x < y)) { r[i] = y; r[l] = x; }
        }
      }
      wave_lds_sync();
    }
  }
  for (uint32_t i = lane; i < c; i += 64) {
    uint32_t w = (uint32_t)(r[i] >> 32);
    if (i > 0 && (uint32_t)(r[i - 1] >> 32) == w) { st.flag[s + i] = 0u; continue; }
    uint32_t cnt = 0;
    float acc = 0.0f;
    for (uint32_t j = i; j < c && (uint32_t)(r[j] >> 32) == w; ++j) {
      ++cnt;
      if (CUSTOM) acc = (float)((double)acc + g.ctab[g.deg[(uint32_t)r[j]]]);
    }
    emit_run<CUSTOM>(g, metric, min_score, u, w, cnt, acc, s + i, st);
  }
  wave_lds_sync();
}

// One workgroup per tile of GT_TILE consecutive sources: the sources with a
// non-empty bucket are compacted into LDS lists by size, then small buckets are
// grouped one per thread (register networks), mid-size ones one per wave
// (LDS bitonic), and large ones are queued for k_group_big.
struct BigItem {
  uint64_t s;
  uint32_t u, c;
};

template <class B, bool CUSTOM>
__global__ __launch_bounds__(NT) void k_group_tiles(GraphView g, B bk, uint64_t ua, uint64_t ub, int metric,
                                                    float min_score, const uint64_t* __restrict__ bucket,
                                                    uint64_t capW, Stage st, BigItem* __restrict__ biglist,
                                                    uint64_t* __restrict__ ctr, uint32_t* __restrict__ zero_a,
                                                    uint32_t* __restrict__ zero_b) {
  // one list per tile: small buckets fill it from the front, mid-size ones from the back
  __shared__ uint32_t l_u[GT_TILE];
  __shared__ uint32_t l_c[GT_TILE];
  __shared__ uint64_t l_s[GT_TILE];
  __shared__ uint32_t n_l[2];
  __shared__ uint64_t wrec[NWAVE][WAVE_MAX];
  const uint64_t W = ctr[C_W];
  if (W > capW || (ctr[C_FLAGS] & F_OVERFLOW)) return;
  const uint64_t nU = ub - ua;
  for (uint64_t t0 = (uint64_t)blockIdx.x * GT_TILE; t0 < nU; t0 += (uint64_t)gridDim.x * GT_TILE) {
    if (threadIdx.x < 2) n_l[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < GT_IPT; ++i) {
      uint64_t u = ua + t0 + (uint64_t)i * NT + threadIdx.x;
      if (u >= ub) continue;
      uint64_t s;
      uint32_t c;
      bk.get(u, s, c);
      if (c == 0) continue;
      if (zero_a) zero_a[u] = 0u;  // leave the bucket counters all-zero for the next call
      if (zero_b) zero_b[u] = 0u;
      if (c <= WAVE_MAX) {
        const int L = c <= SMALL_MAX ? 0 : 1;
        uint32_t k = atomicAdd(&n_l[L], 1u);
        if (L) k = GT_TILE - 1 - k;
        l_u[k] = (uint32_t)u;
        l_c[k] = c;
        l_s[k] = s;
      } else {
        unsigned long long k = atomicAdd((unsigned long long*)&ctr[C_NBIG], 1ull);
        biglist[k] = BigItem{s, (uint32_t)u, c};
      }
    }
    __syncthreads();
    const uint32_t na = n_l[0], nb = n_l[1];
    for (uint32_t j = threadIdx.x; j < na; j += NT) {
      const uint32_t u = l_u[j], c = l_c[j];
      const uint64_t s = l_s[j];
      if (c == 1) {
        uint64_t r = bucket[s];
        float acc = CUSTOM ? (float)((double)0.0f + g.ctab[g.deg[(uint32_t)r]]) : 0.0f;
        emit_run<CUSTOM>(g, metric, min_score, u, (uint32_t)(r >> 32), 1u, acc, s, st);
      } else if (c <= 4) {
        group_small<4, CUSTOM>(g, metric, min_score, u, bucket, s, c, st);
      } else if (c <= 8) {
        group_small<8, CUSTOM>(g, metric, min_score, u, bucket, s, c, st);
      } else {
        group_small<16, CUSTOM>(g, metric, min_score, u, bucket, s, c, st);
      }
    }
    for (uint32_t j = wave_id(); j < nb; j += NWAVE)
      group_wave<CUSTOM>(g, metric, min_score, l_u[GT_TILE - 1 - j], bucket, l_s[GT_TILE - 1 - j],
                         l_c[GT_TILE - 1 - j], wrec[wave_id()], st);
    __syncthreads();
  }
}

// One workgroup per big bucket: LDS bitonic sort, then every thread walks the
// runs that start in its strided slots.
template <bool CUSTOM>
__global__ __launch_bounds__(NT) void k_group_big(GraphView g, int metric, float min_score,
                                                  const uint64_t* __restrict__ bucket, Stage st,
                                                  const BigItem* __restrict__ biglist, uint64_t* __restrict__ ctr) {
  __shared__ uint64_t rec[BIG_CAP];
  const uint64_t nbig = ctr[C_NBIG];
  for (uint64_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    const BigItem it = biglist[b];
    const uint32_t u = it.u, c = it.c;
    const uint64_t s = it.s;
    if (c > BIG_CAP) {
      if (threadIdx.x == 0) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_TOOBIG);
      continue;
    }
    uint32_t n2 = 64;
    while (n2 < c) n2 <<= 1;
    for (uint32_t i = threadIdx.x; i < n2; i += NT) rec[i] = i < c ? bucket[s + i] : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= n2; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = threadIdx.x; i < n2; i += NT) {
          uint32_t l = i ^ j;
          if (l > i) {
            bool up = (i & k) == 0;
            uint64_t x = rec[i], y = rec[l];
            if (up ? (x > y) : (x < y)) { rec[i] = y; rec[l] = x; }
          }
        }
        __syncthreads();
      }
    }
    for (uint32_t i = threadIdx.x; i < c; i += NT) {
      uint32_t w = (uint32_t)(rec[i] >> 32);
      if (i > 0 && (uint32_t)(rec[i - 1] >> 32) == w) { st.flag[s + i] = 0u; continue; }
      uint32_t cnt = 0;
      float acc = 0.0f;
      for (uint32_t j = i; j < c && (uint32_t)(rec[j] >> 32) == w; ++j) {
        ++cnt;
        if (CUSTOM) acc = (float)((double)acc + g.ctab[g.deg[(uint32_t)rec[j]]]);
      }
      emit_run<CUSTOM>(g, metric, min_score, u, w, cnt, acc, s + i, st);
    }
    __syncthreads();
  }
}

// Zero a per-call state arena and set its counters (one launch instead of a
// memset plus a host-to-device copy).
struct CtrInit {
  uint64_t v[NCTR];
};
__global__ void k_arena_init(uint64_t* __restrict__ base, uint64_t words, CtrInit init) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
    base[i] = i < NCTR ? init.v[i] : 0ull;
}

// ctr[dst] = ctr[src] unless it exceeds cap or the overflow flag is set (then 0):
// the length of a scan that must not run past its buffers.
__global__ void k_clamp_n(uint64_t* ctr, uint64_t src, uint64_t cap, uint64_t dst) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t v = ctr[src];
    ctr[dst] = (v > cap || (ctr[C_FLAGS] & F_OVERFLOW)) ? 0 : v;
  }
}

// 32-bit keys for the ascending onesweep sort that orders scores descending.
__global__ void k_desc_keys32(const uint32_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ k,
                              uint32_t* __restrict__ idx) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    k[i] = ~key[i];
    idx[i] = (uint32_t)i;
  }
}

// Compaction of staged candidates (bucket order = u asc, w asc) into the
// candidate buffer at ctr[C_CBASE]; counts NaN candidates.
struct F_Compact {
  Stage st;
  uint32_t* ckey;
  uint32_t* cu;
  uint32_t* cw;
  float* cs;
  const uint64_t* ctr;
  uint64_t* nan_ctr;
  __device__ uint64_t count(uint64_t i) const { return st.flag[i]; }
  __device__ uint64_t count_a(uint64_t i) const { return st.flag[i]; }
  __device__ uint64_t count_b(uint64_t i) const { return st.flag[i]; }
  __device__ void emit(uint64_t i, uint64_t off, uint64_t c) const {
    if (!c) return;
    uint64_t p = ctr[C_CBASE] + off;
    uint32_t k = st.key[i];
    ckey[p] = k;
    cu[p] = st.u[i];
    cw[p] = st.w[i];
    cs[p] = st.s[i];
    if (k == 0) atomicAdd((unsigned long long*)nan_ctr, 1ull);
  }
};

}  // namespace nlp
