// kernels.hpp -- the link-prediction hot path on gfx950.
//
// Reference: /root/reference/inc/predict.hxx.  The reference scans, per source
// vertex u (predict.hxx:287-288), every first-hop neighbour v (hub filter
// deg(v) > MINDEGREE1 skips, predict.hxx:298-301), every second-hop w > u
// (predict.hxx:153-179, ft 292-296), accumulating a per-thread dense counter,
// zeroes u and N(u) (306-307) and scores each touched w (309-311).
//
// Here the same multiset of wedges (u, v, w) is materialised as 64-bit keys
// (u << 32 | w) in an order in which, for every (u, w), the wedges appear with
// v ascending (= the reference's position order in the sorted list N(u)); a
// STABLE radix sort groups them by (u, w) and a segmented pass produces the
// count (basic metrics) or the sequential float accumulation (AA/RA) exactly
// as the reference computes it.  Two generators:
//   path 1 (intermediate-centric, LHub): for v with 0 < deg(v) <= H, for u in
//          the transposed list I(v), the w in N(v) with w > u;
//   path 2 (source-centric, any H, chunked by source range): for u, for v in
//          N(u) surviving the hub filter, the w in N(v) with w > u.
#pragma once
#include "prims.hpp"

namespace nlp {

enum { M_CN = 0, M_JAC, M_SOR, M_SAL, M_HPI, M_HDI, M_LHN, M_AA, M_RA };

__device__ __forceinline__ uint32_t score_key(float s) {
  if (s != s) return 0u;            // NaN ranks last (nlp_oracle.c nlpo_score_key)
  if (s == 0.0f) s = 0.0f;          // -0 == +0
  uint32_t b = __float_as_uint(s);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Basic-metric scores, predict.hxx:504-749.  Degrees are size_t in the
// reference (Graph.hxx:167) -> u64 here, counts are K = uint32_t.
__device__ __forceinline__ float score_basic(int m, uint32_t c, uint64_t du, uint64_t dw) {
  const float fc = (float)c;
  switch (m) {
    case M_CN: return fc;
    case M_JAC: return fc / (float)(du + dw - (uint64_t)c);   // size_t wrap kept
    case M_SOR: return fc / (float)(du + dw);
    case M_SAL: return (float)((double)fc / sqrt((double)(du * dw)));
    case M_HPI: return fc / (float)(du < dw ? du : dw);
    case M_HDI: return fc / (float)(du < dw ? dw : du);
    case M_LHN: return fc / (float)(du * dw);
  }
  return 0.0f;
}

// ---------------------------------------------------------------- edge membership table
// The first-order exclusion (predict.hxx:306-307) asks, for a candidate (u, w)
// with w > u, whether w is in N(u).  A search of the sorted list costs
// log(deg) dependent loads; this table answers with one 64-byte line.  Built
// once per graph (hashpath.hpp k_etab_insert): open addressing over buckets of 8 u64 keys
// (u << 32 | w), one bucket = one cache line, linear probing by bucket, at most
// half full.  Only entries with w > u are stored (a candidate always has
// w > u); duplicate entries (the reference's multiset rows) are stored once.
constexpr uint64_t ET_EMPTY = ~0ull;  // u = 0xffffffff never occurs (span <= 2^32 - 1)
constexpr int ET_SLOTS = 8;

__device__ __forceinline__ uint64_t et_mix(uint64_t x) {  // murmur3 finaliser
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ bool et_has(const uint64_t* __restrict__ tab, uint32_t bits, uint32_t u, uint32_t w) {
  const uint64_t key = ((uint64_t)u << 32) | w;
  const uint64_t mask = (1ull << bits) - 1;
  uint64_t b = et_mix(key) >> (64 - bits);
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const ulonglong2* p = (const ulonglong2*)(tab + b * ET_SLOTS);
    const ulonglong2 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    const uint64_t s[ET_SLOTS] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
    bool hit = false, open = false;
#pragma unroll
    for (int i = 0; i < ET_SLOTS; ++i) {
      hit |= s[i] == key;
      open |= s[i] == ET_EMPTY;
    }
    if (hit) return true;
    if (open) return false;
    b = (b + 1) & mask;
  }
  return false;
}

// et_has for N keys at once: the first buckets of all N are loaded before any
// is compared (one round trip for the N instead of N dependent ones); a key
// whose first bucket is full without it probes on (rare at half load).
__device__ __forceinline__ bool et_has_from(const uint64_t* __restrict__ tab, uint32_t bits, uint64_t key, uint64_t b) {
  const uint64_t mask = (1ull << bits) - 1;
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const ulonglong2* p = (const ulonglong2*)(tab + b * ET_SLOTS);
    const ulonglong2 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    const uint64_t s[ET_SLOTS] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
    bool hit = false, open = false;
#pragma unroll
    for (int i = 0; i < ET_SLOTS; ++i) {
      hit |= s[i] == key;
      open |= s[i] == ET_EMPTY;
    }
    if (hit) return true;
    if (open) return false;
    b = (b + 1) & mask;
  }
  return false;
}
template <int N>
__device__ __forceinline__ void et_has_n(const uint64_t* __restrict__ tab, uint32_t bits, const uint64_t (&key)[N],
                                         const bool (&act)[N], bool (&res)[N]) {
  ulonglong2 q[N][4];
  uint64_t b[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    b[i] = et_mix(key[i]) >> (64 - bits);
    const ulonglong2* p = (const ulonglong2*)(tab + (act[i] ? b[i] : 0ull) * ET_SLOTS);
#pragma unroll
    for (int j = 0; j < 4; ++j) q[i][j] = act[i] ? p[j] : make_ulonglong2(ET_EMPTY, ET_EMPTY);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    bool hit = false, open = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hit |= q[i][j].x == key[i] || q[i][j].y == key[i];
      open |= q[i][j].x == ET_EMPTY || q[i][j].y == ET_EMPTY;
    }
    res[i] = act[i] && (hit || (!open && et_has_from(tab, bits, key[i], (b[i] + 1) & ((1ull << bits) - 1))));
  }
}

// number of entries <= x in the sorted list a[0..n)
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t* __restrict__ a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ bool contains_u32(const uint32_t* __restrict__ a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo < n && a[lo] == x;
}

// Membership in a sorted array with 8-way splits: each round trip issues 7
// independent pivot loads, so a lookup in a hub's adjacency costs about
// log8(n) + 1 dependent loads instead of log2(n) (the loads, not the
// compares, are what a latency-bound scoring thread waits on).
__device__ __forceinline__ bool contains_u32_k8(const uint32_t* __restrict__ a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;  // the lower bound of x lies in [lo, hi]
  while (hi - lo > 8) {
    const uint32_t step = (hi - lo + 7) / 8;
    uint32_t piv[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const uint32_t idx = lo + (uint32_t)(j + 1) * step;
      piv[j] = idx < hi ? a[idx] : 0xffffffffu;
    }
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 7; ++j) c += (lo + (uint32_t)(j + 1) * step < hi && piv[j] < x) ? 1u : 0u;
    const uint32_t nlo = c ? lo + c * step + 1 : lo;
    const uint32_t p = lo + (c + 1) * step;
    hi = (c < 7 && p < hi) ? p : hi;
    lo = nlo;
  }
  bool f = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t idx = lo + (uint32_t)j;
    f |= idx < hi && a[idx] == x;
  }
  return f || (hi < n && a[hi] == x);
}

// ---------------------------------------------------------------- graph build
__global__ void k_degrees(const uint64_t* __restrict__ off, uint64_t span, uint32_t* __restrict__ deg,
                          uint32_t* __restrict__ maxdeg, uint32_t* __restrict__ bad) {
  uint32_t mx = 0;  // the wave's maximum: one atomic per wave, not per row (C4: 9 ms of contended atomics)
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < span; u += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t a = off[u], b = off[u + 1];
    if (b < a) { atomicOr(bad, 1u); deg[u] = 0; continue; }
    uint64_t d = b - a;
    if (d > 0xffffffffull) { atomicOr(bad, 2u); d = 0xffffffffull; }
    deg[u] = (uint32_t)d;
    mx = (uint32_t)d > mx ? (uint32_t)d : mx;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = __shfl_xor(mx, o, 64);
    mx = y > mx ? y : mx;
  }
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(maxdeg, mx);
}

// The AA / RA tables' sparse part: bit d of `present` for every degree d >=
// d0 that some vertex has (the host computes those entries only, glibc's log
// being the reference's), and the scatter of the computed entries.
__global__ void k_deg_present(const uint32_t* __restrict__ deg, uint64_t span, uint32_t d0,
                              unsigned long long* __restrict__ present) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < span; u += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = deg[u];
    if (d >= d0) atomicOr(&present[d >> 6], 1ull << (d & 63));
  }
}
__global__ void k_ctab_scatter(const uint32_t* __restrict__ ds, const double* __restrict__ va,
                               const double* __restrict__ vr, uint64_t n, double* __restrict__ aa,
                               double* __restrict__ ra) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    aa[ds[i]] = va[i];
    ra[ds[i]] = vr[i];
  }
}

// keys must be < span and sorted ascending inside each row.  A descent
// keys[e + 1] < keys[e] is legal only where e + 1 starts a row, so the
// descents over all entries (desc[0], counted here) must equal the descents at
// the starts of non-empty rows (desc[1], k_row_descents): two streaming counts
// instead of a search of the offsets at every descent.
__global__ void k_check_keys(const uint32_t* __restrict__ keys, uint64_t span, uint64_t nnz, uint32_t* __restrict__ bad,
                             unsigned long long* __restrict__ desc) {
  uint64_t c = 0;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[e];
    if (k >= span) atomicOr(bad, 4u);
    if (e + 1 < nnz && keys[e + 1] < k) ++c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&desc[0], (unsigned long long)c);
}

__global__ void k_row_descents(const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys, uint64_t span,
                               uint64_t nnz, unsigned long long* __restrict__ desc) {
  uint64_t c = 0;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < span; u += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = off[u];
    // one non-empty row starts at a position (offsets not yet validated: reads stay below nnz)
    if (a > 0 && a < nnz && off[u + 1] > a && keys[a] < keys[a - 1]) ++c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&desc[1], (unsigned long long)c);
}

// I(v) from the (v << 32 | u) keys sorted by v (u ascending inside a v, the
// keys having been generated in CSR order and sorted stably): tkeys = the u
// halves, toff[x] = the first position whose v >= x (S + 1 entries; item M
// closes the columns above the last v) -- one streaming pass instead of an
// atomic column count plus a scan
__global__ void k_toff_split(const uint64_t* __restrict__ sorted, uint64_t M, uint64_t S, uint64_t* __restrict__ toff,
                             uint32_t* __restrict__ tkeys) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= M; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t v = S;
    if (i < M) {
      const uint64_t x = sorted[i];
      v = x >> 32;
      tkeys[i] = (uint32_t)x;
    }
    const uint64_t vp = i ? (sorted[i - 1] >> 32) + 1 : 0;  // the first column not opened before i
    for (uint64_t c = vp; c <= v; ++c) toff[c] = i;
  }
}

__global__ void k_diff_u64(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint64_t n, uint32_t* __restrict__ flag) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (uint64_t)gridDim.x * blockDim.x)
    if (a[e] != b[e]) { *flag = 1u; return; }
}

__global__ void k_diff_u32(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint64_t n, uint32_t* __restrict__ flag) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (uint64_t)gridDim.x * blockDim.x)
    if (a[e] != b[e]) { *flag = 1u; return; }
}

// ---------------------------------------------------------------- path 1: intermediate-centric
// c[v] = |I(v)| if v survives the hub filter (0 < deg v <= H), else 0.
__global__ void k_p1_vcount(const uint32_t* __restrict__ deg, const uint64_t* __restrict__ toff, uint64_t span,
                            uint32_t H, uint32_t* __restrict__ c) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < span; v += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t d = deg[v];
    c[v] = (d > 0 && d <= H) ? (uint32_t)(toff[v + 1] - toff[v]) : 0u;
  }
}

// One thread per in-edge slot e (v from the scanned per-v counts).
// ewc[e] = #{w in N(v) : w > u} if u in [ua, ub) else 0; efirst[e] = index in N(v)
// of the first such w.
__global__ void k_p1_inedges(const uint64_t* __restrict__ ioff, uint64_t span, const uint64_t* __restrict__ d_E,
                             const uint64_t* __restrict__ toff, const uint32_t* __restrict__ tkeys,
                             const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                             const uint32_t* __restrict__ deg, uint64_t ua, uint64_t ub,
                             uint32_t* __restrict__ ev, uint32_t* __restrict__ eu, uint32_t* __restrict__ ewc,
                             uint32_t* __restrict__ efirst) {
  const uint64_t E = *d_E;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t v = lbs_find(ioff, span, e);
    uint32_t u = tkeys[toff[v] + (e - ioff[v])];
    uint32_t d = deg[v];
    uint32_t first = upper_bound_u32(keys + off[v], d, u);
    ev[e] = (uint32_t)v;
    eu[e] = u;
    efirst[e] = first;
    ewc[e] = (u >= ua && u < ub) ? d - first : 0u;
  }
}

// ---------------------------------------------------------------- path 2: source-centric
// The row of adjacency entry e: the per-graph tile table (tile_row[t] = the
// row of entry t * tile, hashpath.hpp k_hp_tile_rows) bounds it to the rows
// between two table entries, a few probes instead of a search of all offsets.
__device__ __forceinline__ uint64_t row_of_entry(const uint64_t* __restrict__ off, const uint32_t* __restrict__ tile_row,
                                                 uint64_t tile, uint64_t M, uint64_t span, uint64_t e) {
  const uint64_t t = e / tile;
  uint64_t lo = tile_row[t];                                       // off[lo] <= e
  uint64_t hi = (t + 1) * tile < M ? (uint64_t)tile_row[t + 1] + 1 : span;  // off[hi] > e
  while (hi - lo > 1) {  // largest u with off[u] <= e
    const uint64_t mid = (lo + hi) >> 1;
    if (off[mid] <= e) lo = mid; else hi = mid;
  }
  return lo;
}

// One thread per edge e in [e0, e1) (relative index e - e0).
__global__ void k_p2_edges(const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                           const uint32_t* __restrict__ deg, uint64_t span, uint64_t e0, uint64_t e1, uint32_t H,
                           uint32_t* __restrict__ ev, uint32_t* __restrict__ eu, uint32_t* __restrict__ ewc,
                           uint32_t* __restrict__ efirst, const uint32_t* __restrict__ tile_row, uint64_t tile,
                           uint64_t M) {
  const uint64_t n = e1 - e0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t e = e0 + i;
    uint32_t u = (uint32_t)row_of_entry(off, tile_row, tile, M, span, e);
    uint32_t v = keys[e];
    uint32_t d = deg[v];
    bool surv = (H == 0) || (d <= H);                     // predict.hxx:301
    uint32_t first = surv ? upper_bound_u32(keys + off[v], d, u) : d;
    ev[i] = v;
    eu[i] = u;
    efirst[i] = first;
    ewc[i] = d - first;
  }
}

// Running maximum edge index whose wedge offset is <= target (for chunking).
__global__ void k_find_chunk_end(const uint64_t* __restrict__ woff, uint64_t E, uint64_t target,
                                 uint64_t* __restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t lo = 0, hi = E;  // first e with woff[e] > target
    while (lo < hi) {
      uint64_t mid = (lo + hi) >> 1;
      if (woff[mid] <= target) lo = mid + 1; else hi = mid;
    }
    *out = lo;
  }
}

// ---------------------------------------------------------------- common: wedge materialisation
// Wedge slot i < W (slot order = (edge slot, w index), the generator's order)
// -> key (u - ubase) << wb | w, and for AA/RA val = deg(v) (contribution
// table).  A workgroup takes WG_TILE consecutive slots: two searches of the
// edge offsets find its window of edges, which is staged in LDS when it fits
// WG_WIN entries, so each slot's edge is an LDS search instead of ~30
// dependent global loads (edges without wedges can widen a window beyond
// WG_WIN: then the global search).
constexpr int WG_IPT = 8;
constexpr uint32_t WG_TILE = NT * WG_IPT;
constexpr uint32_t WG_WIN = 2048;

template <bool VAL>
__global__ __launch_bounds__(NT) void k_wedges(const uint64_t* __restrict__ woff, uint64_t E,
                                               const uint64_t* __restrict__ d_W, uint64_t wbase,
                                               const uint32_t* __restrict__ ev, const uint32_t* __restrict__ eu,
                                               const uint32_t* __restrict__ efirst, const uint64_t* __restrict__ off,
                                               const uint32_t* __restrict__ keys, const uint32_t* __restrict__ deg,
                                               uint64_t* __restrict__ wkey, uint32_t* __restrict__ wval, uint32_t ubase,
                                               int wb) {
  __shared__ uint64_t s_wo[WG_WIN + 1];
  __shared__ uint32_t s_v[WG_WIN], s_u[WG_WIN], s_f[WG_WIN];
  __shared__ uint64_t s_e[2];
  const uint64_t W = *d_W - wbase;
  const int t = threadIdx.x;
  for (uint64_t t0 = (uint64_t)blockIdx.x * WG_TILE; t0 < W; t0 += (uint64_t)gridDim.x * WG_TILE) {
    const uint64_t t1 = t0 + WG_TILE < W ? t0 + WG_TILE : W;
    if (t < 2) s_e[t] = lbs_find(woff, E, wbase + (t == 0 ? t0 : t1 - 1));
    __syncthreads();
    const uint64_t e_lo = s_e[0], e_hi = s_e[1];
    const uint64_t nw = e_hi - e_lo + 1;
    const bool staged = nw <= WG_WIN;
    if (staged)
      for (uint32_t i = t; i <= nw; i += NT) {
        s_wo[i] = i < nw ? woff[e_lo + i] : (e_lo + nw < E ? woff[e_lo + nw] : ~0ull);
        if (i < nw) {
          s_v[i] = ev[e_lo + i];
          s_u[i] = eu[e_lo + i];
          s_f[i] = efirst[e_lo + i];
        }
      }
    __syncthreads();
    uint32_t v[WG_IPT], u[WG_IPT];
    uint64_t pos[WG_IPT];
    bool ok[WG_IPT];
#pragma unroll
    for (int q = 0; q < WG_IPT; ++q) {
      const uint64_t i = t0 + (uint64_t)q * NT + t;
      ok[q] = i < t1;
      const uint64_t sl = wbase + (ok[q] ? i : t0);
      if (staged) {
        uint32_t lo = 0, hi = (uint32_t)nw;  // last window edge with s_wo <= sl
        while (hi - lo > 1) {
          const uint32_t m = (lo + hi) >> 1;
          if (s_wo[m] <= sl) lo = m; else hi = m;
        }
        v[q] = s_v[lo];
        u[q] = s_u[lo];
        pos[q] = (uint64_t)s_f[lo] + (sl - s_wo[lo]);
      } else {
        const uint64_t e = lbs_find(woff, E, sl);
        v[q] = ev[e];
        u[q] = eu[e];
        pos[q] = (uint64_t)efirst[e] + (sl - woff[e]);
      }
    }
    uint64_t ov[WG_IPT];
#pragma unroll
    for (int q = 0; q < WG_IPT; ++q) ov[q] = off[v[q]];  // in flight together
    uint32_t w[WG_IPT], d[WG_IPT];
#pragma unroll
    for (int q = 0; q < WG_IPT; ++q) {
      w[q] = keys[ov[q] + pos[q]];
      d[q] = VAL ? deg[v[q]] : 0u;
    }
#pragma unroll
    for (int q = 0; q < WG_IPT; ++q) {
      if (!ok[q]) continue;
      const uint64_t i = t0 + (uint64_t)q * NT + t;
      wkey[i] = ((uint64_t)(u[q] - ubase) << wb) | w[q];  // (u - ubase, w) packed: fewer sort digits
      if (VAL) wval[i] = d[q];
    }
    __syncthreads();
  }
}

__global__ void k_run_flags(const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ flag) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    flag[i] = (i == 0 || key[i] != key[i - 1]) ? 1u : 0u;
}

__global__ void k_run_starts(const uint32_t* __restrict__ flag, const uint64_t* __restrict__ rid, uint64_t n,
                             uint64_t* __restrict__ rstart, const uint64_t* __restrict__ d_R) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) rstart[rid[i]] = i;
  if (blockIdx.x == 0 && threadIdx.x == 0) rstart[*d_R] = n;
}

// One thread per candidate run: count / ordered accumulation, first-order
// exclusion (predict.hxx:306-307), score (fs), score <= minScore filter (311).
template <bool CUSTOM>
__global__ void k_score(const uint64_t* __restrict__ rstart, const uint64_t* __restrict__ d_R,
                        const uint64_t* __restrict__ wkey, const uint32_t* __restrict__ wval,
                        const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                        const uint32_t* __restrict__ deg, const double* __restrict__ ctab, int metric,
                        float min_score, uint32_t* __restrict__ ckey, uint32_t* __restrict__ cu,
                        uint32_t* __restrict__ cw, float* __restrict__ cs, uint32_t* __restrict__ cflag,
                        uint32_t maxf2, const uint64_t* __restrict__ etab, uint32_t etbits, uint32_t ubase,
                        int wb) {
  const uint64_t R = *d_R;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t s = rstart[r], e = rstart[r + 1];
    uint64_t k = wkey[s];
    uint32_t u = (uint32_t)(k >> wb) + ubase, w = (uint32_t)(k & ((1ull << wb) - 1));
    bool excl = etab ? et_has(etab, etbits, u, w) : contains_u32(keys + off[u], deg[u], w);
    float sc;
    if (CUSTOM) {
      float acc = 0.0f;  // entry += 1.0/log(deg v) | 1.0/deg v, in v order
      if (!excl)
        for (uint64_t i = s; i < e; ++i) acc = (float)((double)acc + ctab[wval[i]]);
      sc = acc;
    } else {
      uint32_t c = excl ? 0u : (uint32_t)(e - s);
      sc = score_basic(metric, c, deg[u], deg[w]);
    }
    // MAXFACTOR2 (predict.hxx:221,295), see f2_drop
    bool keep = !(sc <= min_score) && !(maxf2 && (uint64_t)deg[w] > (uint64_t)maxf2 * (uint64_t)deg[u]);
    ckey[r] = score_key(sc);
    cu[r] = u;
    cw[r] = w;
    cs[r] = sc;
    cflag[r] = keep ? 1u : 0u;
  }
}

// Compact flagged candidates to base + pos.
__global__ void k_compact_cands(const uint32_t* __restrict__ flag, const uint64_t* __restrict__ pos,
                                const uint64_t* __restrict__ d_n, const uint32_t* __restrict__ ikey,
                                const uint32_t* __restrict__ iu, const uint32_t* __restrict__ iw,
                                const float* __restrict__ is, uint64_t base, uint32_t* __restrict__ okey,
                                uint32_t* __restrict__ ou, uint32_t* __restrict__ ow, float* __restrict__ os) {
  const uint64_t n = *d_n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (flag[i]) {
      uint64_t p = base + pos[i];
      okey[p] = ikey[i];
      ou[p] = iu[i];
      ow[p] = iw[i];
      os[p] = is[i];
    }
  }
}

__global__ void k_count_key0(const uint32_t* __restrict__ key, uint64_t n, unsigned long long* __restrict__ cnt) {
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += key[i] == 0u;
  if (c) atomicAdd(cnt, (unsigned long long)c);
}

// ---------------------------------------------------------------- selection
// tie[i] = key == kth
__global__ void k_tie_flags(const uint32_t* __restrict__ key, uint64_t n, const uint64_t* __restrict__ sel,
                            uint32_t* __restrict__ tie) {
  const uint32_t kth = (uint32_t)sel[3];
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    tie[i] = key[i] == kth ? 1u : 0u;
}

// keep = key > kth, or a tie whose rank (in input order) is < quota.
__global__ void k_keep_flags(const uint32_t* __restrict__ key, uint64_t n, const uint64_t* __restrict__ sel,
                             const uint64_t* __restrict__ trank, uint32_t* __restrict__ keep) {
  const uint32_t kth = (uint32_t)sel[3];
  const uint64_t quota = sel[1];
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t k = key[i];
    keep[i] = (k > kth || (k == kth && trank[i] < quota)) ? 1u : 0u;
  }
}

// 64-bit sort keys for a descending stable sort of u32 keys: ~key.
__global__ void k_desc_keys(const uint32_t* __restrict__ key, uint64_t n, uint64_t* __restrict__ k64,
                            uint32_t* __restrict__ idx) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    k64[i] = (uint64_t)(~key[i]);
    idx[i] = (uint32_t)i;
  }
}

struct EdgeOut {
  uint32_t u, v;
  float score;
};

// ---------------------------------------------------------------- evaluation (main.cxx:48-57)
// |insertions1 ∩ deletions0|: both directions of every predicted link looked
// up in the sorted directed deletion keys (u << 32 | v).
__global__ void k_count_common(const EdgeOut* __restrict__ e, uint64_t n, const uint64_t* __restrict__ keys,
                               uint64_t nk, unsigned long long* __restrict__ common) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const EdgeOut x = e[i];
    const uint64_t a = ((uint64_t)x.u << 32) | x.v, b = ((uint64_t)x.v << 32) | x.u;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint64_t k = q ? b : a;
      uint64_t lo = 0, hi = nk;
      while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if (keys[m] < k) lo = m + 1; else hi = m;
      }
      c += (lo < nk && keys[lo] == k) ? 1 : 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(common, c);
}


__global__ void k_gather_edges(const uint32_t* __restrict__ idx, uint64_t n, const uint32_t* __restrict__ cu,
                               const uint32_t* __restrict__ cw, const float* __restrict__ cs,
                               EdgeOut* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t j = idx[i];
    EdgeOut o;
    o.u = cu[j];
    o.v = cw[j];
    o.score = cs[j];
    out[i] = o;
  }
}

__global__ void k_split_edges(const EdgeOut* __restrict__ in, uint64_t n, uint32_t* __restrict__ ckey,
                              uint32_t* __restrict__ cu, uint32_t* __restrict__ cw, float* __restrict__ cs) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    EdgeOut e = in[i];
    ckey[i] = score_key(e.score);
    cu[i] = e.u;
    cw[i] = e.v;
    cs[i] = e.score;
  }
}

}  // namespace nlp
