// sortpath.hpp -- the sync-free intermediate-centric path with sort grouping.
//
// predict.hxx:292-312 walks, for every source u, the neighbours v that pass
// the hub filter (deg v <= MINDEGREE1, predict.hxx:301) and their neighbours
// w > u (predict.hxx:221), accumulating a per-u counter table.  Here the same
// wedges (u, v, w) are produced from the intermediate side and grouped by a
// sort instead of a table:
//
//   k_sp_survivors  one streaming read of deg[]: the surviving intermediates v,
//                   compacted in ascending v (single-pass scan)
//   k_sp_expand     one thread per survivor: its wedges as records
//                   key = (u - ua) << wbits | w, value = v (single-pass scan,
//                   records land in ascending v)
//   k_sp_hist/pass  stable LSD radix sort of the records by key, 8-bit digits
//                   (onesweep: one histogram launch + one launch per digit).
//                   Stability keeps v ascending inside each (u, w) run, which is
//                   the reference's accumulation order for the Adamic-Adar and
//                   Resource-Allocation sums (predict.hxx:788,828).
//   k_sp_scan<F_Runs> one (u, w) run -> one candidate: first-order exclusion
//                   (predict.hxx:306-307), score, score <= minScore filter
//                   (predict.hxx:311); compacted in (u, w) order
//   k_sp_hist/pass  stable sort of the candidates by score key descending, so the
//                   order is canonical (score desc, u asc, w asc)
//   k_sp_gather     the first min(k, C) candidates -> the caller's edge array
//
// Every launch reads its sizes from device counters; the host enqueues the
// whole chain and synchronises once.  Work is O(S) for the survivor scan and
// O(W) afterwards -- no per-source arrays, so a small wedge count stays cheap
// on a large graph.
//
// Inter-workgroup hand-offs: the single-pass scans use blockIdx-ordered tiles
// in a persistent loop whose grid never exceeds the number of co-resident
// workgroups (the host sizes it from the occupancy query), so every tile a
// look-back waits on is running or done.  Spins are bounded and report
// through the error word like lookback.hpp.
#pragma once
#include "select.hpp"

namespace nlp {

enum { C_WSORT = 11 };  // wedge records to sort (0 after a capacity overflow)

// Arena (u64 words): counters [0, 16), digit histograms, look-back descriptors.
constexpr uint64_t SP_HREC = 16;               // 8 x 256 u32: record-key digits
constexpr uint64_t SP_HORD = SP_HREC + 1024;   // 4 x 256 u32: score-key digits
constexpr uint64_t SP_DESC = SP_HORD + 512;    // descriptors follow

constexpr int SV_STEPS = 32;                   // survivor scan: 64-vertex steps per wave
constexpr int SV_TILE = NT * SV_STEPS;         // 8192 vertices per tile
constexpr int EX_TILE = NT;                    // expansion: one survivor per thread
constexpr int RN_IPT = 4;
constexpr int RN_TILE = NT * RN_IPT;           // run scoring: 1024 records per tile
constexpr int OS2_IPT = 16;
constexpr int OS2_TILE = NT * OS2_IPT;         // onesweep: 4096 keys per tile
constexpr int OS2_LBR = 16;                    // predecessors read per look-back round trip
constexpr uint64_t SP_MAX_N = (1ull << 30) - 1;  // u32 onesweep descriptors: 30-bit values

// Look-back of one wave over 64*R predecessors per round trip (lane l reads
// tiles base-lR .. base-lR-R+1).  Returns the exclusive prefix (wave 0 of the
// workgroup calls it; the value is valid in every lane).
template <int R>
__device__ __forceinline__ uint64_t lb_lookback_r(uint64_t* desc, uint64_t tile, uint64_t agg, uint32_t* err) {
  const int lane = lane_id();
  if (tile == 0) {
    if (lane == 0) lb_store(&desc[0], LB_PFX | agg);
    return 0;
  }
  if (lane == 0) lb_store(&desc[tile], LB_AGG | agg);
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  uint32_t spins = 0;
  while (true) {
    uint64_t d[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t j = base - (int64_t)(lane * R + r);
      d[r] = j >= 0 ? lb_load(&desc[j]) : LB_PFX;  // before tile 0: prefix 0
    }
    uint64_t sum = 0;
    bool found = false, wait = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!found) {
        const uint64_t s = d[r] & ~LB_VAL;
        wait |= s == 0;
        sum += d[r] & LB_VAL;
        found = s == LB_PFX;
      }
    }
    const uint64_t pf = __ballot(found);
    const int first = pf ? __ffsll((long long)pf) - 1 : 63;
    const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);  // lanes 0..first
    if (__ballot(wait) & need) {
      if (++spins > LB_SPIN_LIMIT) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t v = lane <= first ? sum : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    excl += v;
    if (pf) break;
    base -= 64 * R;
  }
  if (lane == 0) lb_store(&desc[tile], LB_PFX | (excl + agg));
  return excl;
}

__device__ __forceinline__ uint64_t lane_mask_lt() {
  const int lane = lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// ---------------------------------------------------------------- survivors
// Tile = 4 waves x 32 steps x 64 consecutive vertices; a vertex survives when
// 1 <= deg v <= H (H = 0: IHub, every vertex with edges).  Output ascending v.
__global__ __launch_bounds__(NT) void k_sp_survivors(const uint32_t* __restrict__ deg, uint64_t S, uint32_t H,
                                                     uint32_t* __restrict__ surv, uint64_t* __restrict__ desc,
                                                     uint64_t* __restrict__ ctr) {
  __shared__ uint64_t s_w[NWAVE];
  __shared__ uint64_t s_excl;
  const int lane = lane_id(), wv = wave_id();
  const uint32_t hm = H ? H : 0xffffffffu;
  const uint64_t ntiles = (S + SV_TILE - 1) / SV_TILE;
  const uint64_t lt = lane_mask_lt();
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t b0 = tile * SV_TILE + (uint64_t)wv * (64 * SV_STEPS) + lane;
    uint32_t dv[SV_STEPS];
#pragma unroll
    for (int i = 0; i < SV_STEPS; ++i) {
      const uint64_t v = b0 + (uint64_t)i * 64;
      dv[i] = v < S ? deg[v] : 0u;
    }
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < SV_STEPS; ++i) bits |= (uint32_t)(dv[i] - 1u < hm) << i;  // 1 <= d <= H
    uint64_t wt = (uint64_t)__popc(bits);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wt += __shfl_xor(wt, o, 64);
    if (lane == 0) s_w[wv] = wt;
    __syncthreads();
    if (wv == 0) {
      uint64_t agg = 0;
#pragma unroll
      for (int w = 0; w < NWAVE; ++w) agg += s_w[w];
      const uint64_t e = lb_lookback_r<4>(desc, tile, agg, err);
      if (lane == 0) {
        s_excl = e;
        if (tile == ntiles - 1) ctr[C_NV] = e + agg;
      }
    }
    __syncthreads();
    uint64_t run = s_excl;
    for (int w = 0; w < wv; ++w) run += s_w[w];
#pragma unroll
    for (int i = 0; i < SV_STEPS; ++i) {
      const bool f = (bits >> i) & 1u;
      const uint64_t m = __ballot(f);
      if (f) surv[run + __popcll(m & lt)] = (uint32_t)(b0 + (uint64_t)i * 64);
      run += __popcll(m);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- wedge records
// One thread per survivor v (ascending): for each in-edge u -> v with u in
// [ua, ub), the wedges (u, v, w) with w in N(v), w > u.  Records beyond capW are
// not written; the total still goes to ctr[C_W] (the host regrows and reruns).
__global__ __launch_bounds__(NT) void k_sp_expand(GraphView g, uint64_t ua, uint64_t ub, int wbits,
                                                  const uint32_t* __restrict__ surv, uint64_t capW,
                                                  uint64_t* __restrict__ rkey, uint32_t* __restrict__ rval,
                                                  uint64_t* __restrict__ desc, uint64_t* __restrict__ ctr) {
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_excl;
  const uint64_t n = ctr[C_NV];
  const uint64_t ntiles = (n + EX_TILE - 1) / EX_TILE;
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t i = tile * EX_TILE + threadIdx.x;
    uint32_t v = 0, d = 0;
    uint64_t a = 0, b = 0, c = 0;
    const uint32_t* nv = g.keys;
    if (i < n) {
      v = surv[i];
      d = g.deg[v];
      a = g.toff[v];
      b = g.toff[v + 1];
      nv = g.keys + g.off[v];
      for (uint64_t j = a; j < b; ++j) {
        const uint32_t u = g.tkeys[j];
        if (u >= ua && u < ub) c += d - upper_bound_u32(nv, d, u);
      }
    }
    uint64_t agg;
    const uint64_t x = block_excl_scan(c, s_red, &agg);
    if (wave_id() == 0) {
      const uint64_t e = lb_lookback_r<4>(desc, tile, agg, err);
      if (lane_id() == 0) {
        s_excl = e;
        if (tile == ntiles - 1) ctr[C_W] = e + agg;
      }
    }
    __syncthreads();
    uint64_t pos = s_excl + x;
    if (c && pos + c <= capW) {
      for (uint64_t j = a; j < b; ++j) {
        const uint32_t u = g.tkeys[j];
        if (u < ua || u >= ub) continue;
        const uint64_t hi = (uint64_t)(u - ua) << wbits;
        for (uint32_t k = upper_bound_u32(nv, d, u); k < d; ++k) {
          rkey[pos] = hi | nv[k];
          rval[pos] = v;
          ++pos;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- onesweep radix sort
// Digit histograms of ndig 8-bit digits in one read.  n = *d_n, or 0 when it
// exceeds cap (then F_OVERFLOW is raised); block 0 stores the effective n.
template <typename K>
__global__ __launch_bounds__(NT) void k_sp_hist(const K* __restrict__ keys, const uint64_t* __restrict__ d_n,
                                                uint64_t cap, int ndig, uint32_t* __restrict__ ghist,
                                                uint64_t* __restrict__ n_out, uint64_t* __restrict__ flags) {
  __shared__ uint32_t h[8][RS_BINS];
  for (int i = threadIdx.x; i < 8 * RS_BINS; i += NT) (&h[0][0])[i] = 0;
  __syncthreads();
  uint64_t n = *d_n;
  if (n > cap) {
    n = 0;
    if (flags && blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long*)flags, F_OVERFLOW);
  }
  if (n_out && blockIdx.x == 0 && threadIdx.x == 0) *n_out = n;
  for (uint64_t j = (uint64_t)blockIdx.x * NT + threadIdx.x; j < n; j += (uint64_t)gridDim.x * NT) {
    const K k = keys[j];
    for (int dd = 0; dd < ndig; ++dd) atomicAdd(&h[dd][(uint32_t)(k >> (8 * dd)) & 0xffu], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ndig * RS_BINS; i += NT) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&ghist[i], c);
  }
}

__device__ __forceinline__ void st_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-digit look-back of digit t: descriptors are u32 {status:2, count:30};
// each round trip reads OS2_LBR predecessors and resumes exactly where a
// not-yet-published one stopped it.
__device__ __forceinline__ uint32_t os2_lookback(uint32_t* desc, uint64_t tile, int t, uint32_t run,
                                                 uint32_t* err) {
  constexpr uint32_t AGG = 1u << 30, PFX = 2u << 30, VAL = AGG - 1;
  uint32_t* my = desc + tile * RS_BINS + t;
  if (tile == 0) {
    st_u32(my, PFX | run);
    return 0;
  }
  st_u32(my, AGG | run);
  uint32_t excl = 0, spins = 0;
  int64_t j = (int64_t)tile - 1;
  while (true) {
    uint32_t x[OS2_LBR];
#pragma unroll
    for (int r = 0; r < OS2_LBR; ++r) x[r] = j - r >= 0 ? ld_u32(desc + (uint64_t)(j - r) * RS_BINS + t) : PFX;
    int used = 0;
    bool done = false, blocked = false;
#pragma unroll
    for (int r = 0; r < OS2_LBR; ++r) {
      if (!done && !blocked) {
        const uint32_t s = x[r] >> 30;
        if (s == 0) {
          blocked = true;
        } else {
          excl += x[r] & VAL;
          ++used;
          done = s == 2;
        }
      }
    }
    if (done) break;
    j -= used;
    if (used == 0) {
      if (++spins > LB_SPIN_LIMIT) {
        atomicOr(err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  st_u32(my, PFX | (excl + run));
  return excl;
}

// One stable counting pass on digit (key >> shift) & 255.  Wave w of a tile owns
// 64*OS2_IPT consecutive keys; ranks come from ballot multisplit plus a per-wave
// running digit count in LDS, so the tile order is preserved exactly.
template <typename K>
__global__ __launch_bounds__(NT) void k_sp_pass(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                const uint64_t* __restrict__ d_n, int shift,
                                                const uint32_t* __restrict__ ghist, uint32_t* __restrict__ desc,
                                                uint32_t* __restrict__ err) {
  constexpr int WT = 64 * OS2_IPT;
  __shared__ uint32_t s_wcnt[NWAVE][RS_BINS];
  __shared__ uint32_t s_base[RS_BINS];
  __shared__ uint64_t s_red[NWAVE + 1];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + OS2_TILE - 1) / OS2_TILE;
  if (blockIdx.x >= ntiles) return;
  uint64_t tot;
  const uint32_t dbase = (uint32_t)block_excl_scan(ghist[t], s_red, &tot);
  const uint64_t lt = lane_mask_lt();
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    for (int i = t; i < NWAVE * RS_BINS; i += NT) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t b0 = tile * OS2_TILE + (uint64_t)wv * WT + lane;
    K k[OS2_IPT];
    uint32_t v[OS2_IPT], dg[OS2_IPT], rk[OS2_IPT];
#pragma unroll
    for (int i = 0; i < OS2_IPT; ++i) {
      const uint64_t j = b0 + (uint64_t)i * 64;
      k[i] = j < n ? kin[j] : (K)0;
      v[i] = j < n ? vin[j] : 0u;
    }
#pragma unroll
    for (int i = 0; i < OS2_IPT; ++i) {
      const bool ok = b0 + (uint64_t)i * 64 < n;
      const uint32_t d = (uint32_t)(k[i] >> shift) & 0xffu;
      dg[i] = d;
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint64_t bb = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bb : ~bb;
      }
      const uint32_t before = ok ? s_wcnt[wv][d] : 0u;
      rk[i] = before + (uint32_t)__popcll(peers & lt);
      wave_lds_sync();
      if (ok && (peers & lt) == 0) s_wcnt[wv][d] = before + (uint32_t)__popcll(peers);
      wave_lds_sync();
    }
    __syncthreads();
    // thread t owns digit t: cross-wave exclusive prefix and the tile count
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) {
      const uint32_t c = s_wcnt[w][t];
      s_wcnt[w][t] = run;
      run += c;
    }
    s_base[t] = dbase + os2_lookback(desc, tile, t, run, err);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < OS2_IPT; ++i) {
      if (b0 + (uint64_t)i * 64 < n) {
        const uint64_t pos = (uint64_t)s_base[dg[i]] + s_wcnt[wv][dg[i]] + rk[i];
        kout[pos] = k[i];
        vout[pos] = v[i];
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- generic single-pass scan
// F: count(i) -> u32 (evaluated once, striped), emit(i, off, c).  Persistent
// blockIdx-ordered tiles; the grand total goes to *total.
template <class F, int IPT>
__global__ __launch_bounds__(NT) void k_sp_scan(F f, const uint64_t* __restrict__ d_n, uint64_t* __restrict__ desc,
                                                uint32_t* __restrict__ err, uint64_t* __restrict__ total) {
  constexpr int TILE = NT * IPT;
  __shared__ uint32_t s_cnt[TILE];
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_excl;
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t base = tile * TILE;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint64_t j = base + (uint64_t)i * NT + threadIdx.x;
      s_cnt[i * NT + threadIdx.x] = j < n ? f.count(j, n) : 0u;
    }
    __syncthreads();
    uint32_t cs[IPT];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      cs[i] = s_cnt[threadIdx.x * IPT + i];
      s += cs[i];
    }
    uint64_t agg;
    const uint64_t texcl = block_excl_scan(s, s_red, &agg);
    if (wave_id() == 0) {
      const uint64_t e = lb_lookback_r<4>(desc, tile, agg, err);
      if (lane_id() == 0) {
        s_excl = e;
        if (tile == ntiles - 1 && total) *total = e + agg;
      }
    }
    uint32_t run = (uint32_t)texcl;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      s_cnt[threadIdx.x * IPT + i] = run;
      run += cs[i];
    }
    __syncthreads();
    const uint64_t tb = s_excl;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int li = i * NT + threadIdx.x;
      const uint64_t j = base + li;
      if (j < n) {
        const uint32_t o = s_cnt[li];
        const uint32_t nx = li + 1 < TILE ? s_cnt[li + 1] : (uint32_t)agg;
        f.emit(j, tb + o, nx - o);
      }
    }
    __syncthreads();
  }
}

// One (u, w) run of the sorted records -> one scored candidate.
template <bool CUSTOM>
struct F_Runs {
  GraphView g;
  int metric;
  float min_score;
  uint64_t ua;
  int wbits;
  const uint64_t* rkey;
  const uint32_t* rval;
  float* stash;  // per record slot: the run's score (read back by emit)
  uint32_t* cu;
  uint32_t* cw;
  float* cs;
  uint32_t* okey;  // ~score_key: ascending sort = score descending
  uint32_t* oval;  // candidate index
  uint64_t* nan_ctr;
  __device__ uint32_t count(uint64_t i, uint64_t n) const {
    const uint64_t k = rkey[i];
    if (i > 0 && rkey[i - 1] == k) return 0u;
    uint32_t c = 1;
    float acc = CUSTOM ? (float)((double)0.0f + g.ctab[g.deg[rval[i]]]) : 0.0f;
    for (uint64_t j = i + 1; j < n && rkey[j] == k; ++j) {
      ++c;
      if (CUSTOM) acc = (float)((double)acc + g.ctab[g.deg[rval[j]]]);
    }
    const uint32_t u = (uint32_t)(ua + (k >> wbits));
    const uint32_t w = (uint32_t)(k & ((1ull << wbits) - 1));
    const bool excl = contains_u32(g.keys + g.off[u], g.deg[u], w);
    float sc;
    if (CUSTOM) sc = excl ? 0.0f : acc;
    else sc = score_basic(metric, excl ? 0u : c, g.deg[u], g.deg[w]);
    stash[i] = sc;
    return !(sc <= min_score) ? 1u : 0u;  // NaN passes
  }
  __device__ void emit(uint64_t i, uint64_t off, uint32_t c) const {
    if (!c) return;
    const uint64_t k = rkey[i];
    const float sc = stash[i];
    cu[off] = (uint32_t)(ua + (k >> wbits));
    cw[off] = (uint32_t)(k & ((1ull << wbits) - 1));
    cs[off] = sc;
    okey[off] = ~score_key(sc);
    oval[off] = (uint32_t)off;
    if (sc != sc) atomicAdd((unsigned long long*)nan_ctr, 1ull);
  }
};

// The first min(k, C) candidates of the score order -> caller's edges.
__global__ __launch_bounds__(NT) void k_sp_gather(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ cu,
                                                  const uint32_t* __restrict__ cw, const float* __restrict__ cs,
                                                  uint64_t k, EdgeOut* __restrict__ out,
                                                  uint64_t* __restrict__ ctr) {
  const uint64_t m = std::min<uint64_t>(ctr[C_C], k);
  if (blockIdx.x == 0 && threadIdx.x == 0) ctr[C_OUT_N] = m;
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (uint64_t)gridDim.x * NT) {
    const uint32_t x = idx[i];
    out[i] = EdgeOut{cu[x], cw[x], cs[x]};
  }
}

}  // namespace nlp
