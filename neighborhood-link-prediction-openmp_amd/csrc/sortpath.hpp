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

// Digit histograms are kept in HCOPIES copies (workgroup b adds into copy
// b % HCOPIES, readers sum the copies): thousands of workgroups adding into one
// 4 KiB histogram serialise on a few cache lines.
constexpr int HCOPIES = 16;
constexpr uint32_t HSTRIDE = 8 * 256;  // u32 per copy: up to 8 digits of 256 bins

// Arena (u64 words): counters [0, 16), digit histograms, look-back descriptors.
constexpr uint64_t SP_HREC = 16;                                 // record-key digits
constexpr uint64_t SP_HORD = SP_HREC + HCOPIES * HSTRIDE / 2;    // score-key digits
constexpr uint64_t SP_DESC = SP_HORD + HCOPIES * HSTRIDE / 2;    // descriptors follow

__device__ __forceinline__ uint32_t* hist_copy(uint32_t* h) { return h + (blockIdx.x % HCOPIES) * HSTRIDE; }
__device__ __forceinline__ uint32_t hist_total(const uint32_t* h, uint32_t i) {
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < HCOPIES; ++c) s += h[c * HSTRIDE + i];
  return s;
}

constexpr int SV_STEPS = 8;                    // survivor scan: 256-vertex steps per wave
constexpr int SV_TILE = NT * 4 * SV_STEPS;     // 8192 vertices per tile
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

// Optional phase stamps for tools/ubench (nullptr in the product): workgroup b
// writes s_memrealtime (100 MHz) of phase i of its first tile to stamp[8 b + i].
__device__ __forceinline__ void sp_stamp(uint64_t* stamp, bool first, int i) {
  if (stamp && first && threadIdx.x == 0) stamp[blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ uint64_t lane_mask_lt() {
  const int lane = lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// ---------------------------------------------------------------- survivors
// Tile = 4 waves x STEPS steps x 256 consecutive vertices (16-byte loads, lane l
// of step i holds vertices base + 256 i + 4 l .. +3); a vertex survives when
// 1 <= deg v <= H (H = 0: IHub, every vertex with edges).  Output ascending v.
template <int STEPS = SV_STEPS>
__global__ __launch_bounds__(NT) void k_sp_survivors(const uint32_t* __restrict__ deg, uint64_t S, uint32_t H,
                                                     uint32_t* __restrict__ surv, uint64_t* __restrict__ desc,
                                                     uint64_t* __restrict__ ctr, uint64_t* __restrict__ stamp) {
  static_assert(STEPS * 4 <= 32, "flag bits");
  constexpr uint64_t TILE = (uint64_t)NT * 4 * STEPS;
  __shared__ uint64_t s_w[NWAVE];
  __shared__ uint64_t s_excl;
  const int lane = lane_id(), wv = wave_id();
  const uint32_t hm = H ? H : 0xffffffffu;
  const uint64_t ntiles = (S + TILE - 1) / TILE;
  const uint64_t lt = lane_mask_lt();
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == blockIdx.x;
    sp_stamp(stamp, first, 0);
    const uint64_t b0 = tile * TILE + (uint64_t)wv * (256 * STEPS) + 4 * (uint64_t)lane;
    uint4 dv[STEPS];
#pragma unroll
    for (int i = 0; i < STEPS; ++i) {
      const uint64_t v = b0 + (uint64_t)i * 256;
      if (v + 3 < S) {
        dv[i] = *(const uint4*)(deg + v);
      } else {
        dv[i].x = v < S ? deg[v] : 0u;
        dv[i].y = v + 1 < S ? deg[v + 1] : 0u;
        dv[i].z = v + 2 < S ? deg[v + 2] : 0u;
        dv[i].w = 0u;
      }
    }
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < STEPS; ++i) {
      bits |= (uint32_t)(dv[i].x - 1u < hm) << (4 * i);
      bits |= (uint32_t)(dv[i].y - 1u < hm) << (4 * i + 1);
      bits |= (uint32_t)(dv[i].z - 1u < hm) << (4 * i + 2);
      bits |= (uint32_t)(dv[i].w - 1u < hm) << (4 * i + 3);
    }
    uint64_t wt = (uint64_t)__popc(bits);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wt += __shfl_xor(wt, o, 64);
    if (lane == 0) s_w[wv] = wt;
    __syncthreads();
    sp_stamp(stamp, first, 1);
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
    sp_stamp(stamp, first, 2);
    uint64_t run = s_excl;
    for (int w = 0; w < wv; ++w) run += s_w[w];
#pragma unroll
    for (int i = 0; i < STEPS; ++i) {
      const uint32_t nib = (bits >> (4 * i)) & 0xfu;
      uint64_t before = 0, stepn = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint64_t m = __ballot((nib >> e) & 1u);
        before += __popcll(m & lt);
        stepn += __popcll(m);
      }
      uint64_t o = run + before;
      const uint64_t v = b0 + (uint64_t)i * 256;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if ((nib >> e) & 1u) surv[o++] = (uint32_t)(v + e);
      run += stepn;
    }
    __syncthreads();
    sp_stamp(stamp, first, 3);
  }
}

// ---------------------------------------------------------------- degree-class index
// Built once per graph: the vertices of degree 1..DCAP grouped by degree, so
// the survivors of any hub threshold H <= DCAP are one contiguous prefix and a
// prediction needs no pass over deg[].  Order inside a class is arbitrary; it
// is used only where the accumulation order of a run cannot matter (the count
// metrics), the Adamic-Adar / Resource-Allocation sums keep k_sp_survivors.
constexpr uint32_t DCAP = 1024;

__global__ __launch_bounds__(NT) void k_deg_class_hist(const uint32_t* __restrict__ deg, uint64_t S,
                                                       uint32_t* __restrict__ hist /*DCAP + 2*/) {
  __shared__ uint32_t h[DCAP + 2];
  for (uint32_t i = threadIdx.x; i < DCAP + 2; i += NT) h[i] = 0;
  __syncthreads();
  for (uint64_t v = (uint64_t)blockIdx.x * NT + threadIdx.x; v < S; v += (uint64_t)gridDim.x * NT)
    atomicAdd(&h[std::min<uint32_t>(deg[v], DCAP + 1)], 1u);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < DCAP + 2; i += NT)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// cursor[d] starts at the first slot of class d (relative to class 1).
__global__ __launch_bounds__(NT) void k_deg_class_scatter(const uint32_t* __restrict__ deg, uint64_t S,
                                                          unsigned long long* __restrict__ cursor,
                                                          uint32_t* __restrict__ vbydeg) {
  for (uint64_t v = (uint64_t)blockIdx.x * NT + threadIdx.x; v < S; v += (uint64_t)gridDim.x * NT) {
    const uint32_t d = deg[v];
    if (d >= 1 && d <= DCAP) vbydeg[atomicAdd(&cursor[d], 1ull)] = (uint32_t)v;
  }
}

// ---------------------------------------------------------------- per-range degree-class index
// A multi-GPU rank predicts one source range [ua, ub) of its graph replica; only
// the intermediates with an in-neighbour u in the range emit wedges.  The
// index of classes 1..H restricted to them is built once per (range, H): pass 1
// counts them per class, the host turns the counts into class starts, pass 2
// scatters them (order inside a class arbitrary, like the full index).
__device__ __forceinline__ bool in_neighbour_in_range(const GraphView& g, uint32_t v, uint64_t ua, uint64_t ub) {
  uint64_t lo = g.toff[v], hi = g.toff[v + 1];
  const uint64_t end = hi;
  while (lo < hi) {  // first u >= ua in the ascending list I(v)
    const uint64_t mid = (lo + hi) >> 1;
    if (g.tkeys[mid] < ua) lo = mid + 1;
    else hi = mid;
  }
  return lo < end && g.tkeys[lo] < ub;
}

template <bool SCATTER>
__global__ __launch_bounds__(NT) void k_range_index(GraphView g, const uint32_t* __restrict__ vbydeg, uint64_t n,
                                                    uint32_t H, uint64_t ua, uint64_t ub,
                                                    unsigned long long* __restrict__ cnt, uint32_t* __restrict__ out) {
  __shared__ uint32_t s_c[DCAP + 1];
  __shared__ unsigned long long s_base[DCAP + 1];
  for (uint64_t base = (uint64_t)blockIdx.x * NT; base < n; base += (uint64_t)gridDim.x * NT) {
    for (uint32_t d = threadIdx.x; d <= H; d += NT) s_c[d] = 0;
    __syncthreads();
    const uint64_t i = base + threadIdx.x;
    uint32_t v = 0, d = 0, slot = 0;
    bool keep = false;
    if (i < n) {
      v = vbydeg[i];
      keep = in_neighbour_in_range(g, v, ua, ub);
      if (keep) {
        d = g.deg[v];
        slot = atomicAdd(&s_c[d], 1u);
      }
    }
    __syncthreads();
    for (uint32_t c = threadIdx.x; c <= H; c += NT)
      if (s_c[c]) s_base[c] = atomicAdd(&cnt[c], (unsigned long long)s_c[c]);
    __syncthreads();
    if (SCATTER && keep) out[s_base[d] + slot] = v;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- wedge records
// One thread per survivor v (ascending): for each in-edge u -> v with u in
// [ua, ub), the wedges (u, v, w) with w in N(v), w > u.  Records beyond capW are
// not written; the total still goes to ctr[C_W] (the host regrows and reruns).
// HIST: also the histogram of record-key digit (key >> hshift) & 255 (the MSD
// pass), accumulated per workgroup in LDS; the last tile stores the sortable
// record count ctr[C_WSORT] (0 and F_OVERFLOW when the records exceed capW).
template <bool HIST>
__global__ __launch_bounds__(NT) void k_sp_expand(GraphView g, uint64_t ua, uint64_t ub, int wbits,
                                                  const uint32_t* __restrict__ surv, uint64_t capW,
                                                  uint64_t* __restrict__ rkey, uint32_t* __restrict__ rval,
                                                  uint64_t* __restrict__ desc, uint64_t* __restrict__ ctr,
                                                  int hshift, uint32_t* __restrict__ ghist, int hdigits = 1) {
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_h[HIST ? 2 * RS_BINS : 1];
  const uint64_t n = ctr[C_NV];
  const uint64_t ntiles = (n + EX_TILE - 1) / EX_TILE;
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  if (blockIdx.x >= ntiles) return;
  if (HIST) {
    s_h[threadIdx.x] = 0;
    s_h[RS_BINS + threadIdx.x] = 0;
    __syncthreads();
  }
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
        if (tile == ntiles - 1) {
          const uint64_t W = e + agg;
          ctr[C_W] = W;
          if (HIST) {
            ctr[C_WSORT] = W <= capW ? W : 0;
            if (W > capW) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_OVERFLOW);
          }
        }
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
          const uint64_t key = hi | nv[k];
          rkey[pos] = key;
          rval[pos] = v;
          if (HIST) {
            atomicAdd(&s_h[(uint32_t)(key >> hshift) & 0xffu], 1u);
            if (hdigits > 1) atomicAdd(&s_h[RS_BINS + ((uint32_t)(key >> (hshift + 8)) & 0xffu)], 1u);
          }
          ++pos;
        }
      }
    }
    __syncthreads();
  }
  if (HIST) {
    uint32_t* hc = hist_copy(ghist);
    for (int dd = 0; dd < hdigits; ++dd) {
      const uint32_t c = s_h[dd * RS_BINS + threadIdx.x];
      if (c) atomicAdd(&hc[dd * RS_BINS + threadIdx.x], c);
    }
  }
}

// ---------------------------------------------------------------- onesweep radix sort
// Digit histograms of ndig 8-bit digits in one read.  n = *d_n, or 0 when it
// exceeds cap (then F_OVERFLOW is raised); block 0 stores the effective n.
template <typename K>
__global__ __launch_bounds__(NT) void k_sp_hist(const K* __restrict__ keys, const uint64_t* __restrict__ d_n,
                                                uint64_t cap, int shift0, int ndig, uint32_t* __restrict__ ghist,
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
    for (int dd = 0; dd < ndig; ++dd) atomicAdd(&h[dd][(uint32_t)(k >> (shift0 + 8 * dd)) & 0xffu], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ndig * RS_BINS; i += NT) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&hist_copy(ghist)[i], c);
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
// Candidate columns for the last ordering pass, which writes the caller's
// edges directly (position < k) instead of the next key/value buffers.
struct GatherOut {
  const uint32_t* cu;
  const uint32_t* cw;
  const float* cs;
  uint64_t k;
  EdgeOut* out;
};

// NEXT_HIST: also count digits 1..3 (shift 8, 16, 24) of the input keys into
// the histogram copies at nhist (the first pass of a 32-bit sort whose later
// histograms were not produced upstream).
template <typename K, int IPT = OS2_IPT, bool GATHER = false, bool NEXT_HIST = false>
__global__ __launch_bounds__(NT) void k_sp_pass(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                const uint64_t* __restrict__ d_n, int shift,
                                                const uint32_t* __restrict__ ghist, uint32_t* __restrict__ desc,
                                                uint32_t* __restrict__ err, uint64_t* __restrict__ stamp,
                                                GatherOut go, uint32_t* __restrict__ nhist = nullptr) {
  constexpr int WT = 64 * IPT;
  __shared__ uint32_t s_wcnt[NWAVE][RS_BINS];
  __shared__ uint32_t s_nh[NEXT_HIST ? 3 : 1][NEXT_HIST ? RS_BINS : 1];
  __shared__ uint32_t s_base[RS_BINS];
  __shared__ uint64_t s_red[NWAVE + 1];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + (NT * IPT) - 1) / (NT * IPT);
  if (blockIdx.x >= ntiles) return;
  uint64_t tot;
  const uint32_t dbase = (uint32_t)block_excl_scan(hist_total(ghist, t), s_red, &tot);
  const uint64_t lt = lane_mask_lt();
  if (NEXT_HIST)
    for (int i = t; i < 3 * RS_BINS; i += NT) (&s_nh[0][0])[i] = 0;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == blockIdx.x;
    sp_stamp(stamp, first, 0);
    for (int i = t; i < NWAVE * RS_BINS; i += NT) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t b0 = tile * (NT * IPT) + (uint64_t)wv * WT + lane;
    K k[IPT];
    uint32_t v[IPT], dg[IPT], rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint64_t j = b0 + (uint64_t)i * 64;
      k[i] = j < n ? kin[j] : (K)0;
      v[i] = j < n ? vin[j] : 0u;
    }
    if (stamp) {  // phase 1 = keys landed
      uint64_t z = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) z |= (uint64_t)k[i] ^ v[i];
      if (z == 0x5a5a5a5a5a5aull) stamp[0] = z;
      sp_stamp(stamp, first, 1);
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
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
    sp_stamp(stamp, first, 2);
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
    sp_stamp(stamp, first, 3);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      if (b0 + (uint64_t)i * 64 < n) {
        const uint64_t pos = (uint64_t)s_base[dg[i]] + s_wcnt[wv][dg[i]] + rk[i];
        if (GATHER) {
          if (pos < go.k) go.out[pos] = EdgeOut{go.cu[v[i]], go.cw[v[i]], go.cs[v[i]]};
        } else {
          kout[pos] = k[i];
          vout[pos] = v[i];
        }
        if (NEXT_HIST) {
#pragma unroll
          for (int dd = 0; dd < 3; ++dd) atomicAdd(&s_nh[dd][(uint32_t)(k[i] >> (8 * dd + 8)) & 0xffu], 1u);
        }
      }
    }
    __syncthreads();
    sp_stamp(stamp, first, 4);
  }
  if (NEXT_HIST) {
    uint32_t* hc = hist_copy(nhist);
    for (int i = t; i < 3 * RS_BINS; i += NT) {
      const uint32_t c = s_nh[i / RS_BINS][i % RS_BINS];
      if (c) atomicAdd(&hc[i], c);
    }
  }
}

// ---------------------------------------------------------------- onesweep pass, general tile shape
// Same contract as k_sp_pass.  NTB threads (256 or 512) x IPT substeps per
// tile.  Per-(substep, wave, digit) counts are written once by the digit
// group's leader lane (no read-modify-write chain inside the ranking loop).
// G = NTB / 256 threads serve each digit: they prefix-sum its counts and read
// LBR predecessors each per look-back round trip (G * LBR per round trip).
template <int G, int LBR>
__device__ __forceinline__ uint32_t osg_lookback(uint32_t* desc, uint64_t tile, int d, int q, uint32_t run,
                                                 uint32_t* err) {
  constexpr uint32_t AGG = 1u << 30, PFX = 2u << 30, VAL = AGG - 1;
  uint32_t* my = desc + tile * RS_BINS + d;
  if (tile == 0) {
    if (q == 0) st_u32(my, PFX | run);
    return 0;
  }
  if (q == 0) st_u32(my, AGG | run);
  const int gl = lane_id() & ~(G - 1);
  uint32_t excl = 0, spins = 0;
  int64_t j = (int64_t)tile - 1;
  while (true) {
    uint32_t x[LBR];
#pragma unroll
    for (int r = 0; r < LBR; ++r) {
      const int64_t jj = j - (int64_t)(q * LBR + r);
      x[r] = jj >= 0 ? ld_u32(desc + (uint64_t)jj * RS_BINS + d) : PFX;
    }
    uint32_t sum = 0;
    int used = 0, state = 0;  // 0 open, 1 reached a prefix, 2 blocked on an unpublished tile
#pragma unroll
    for (int r = 0; r < LBR; ++r) {
      if (state == 0) {
        const uint32_t st = x[r] >> 30;
        if (st == 0) {
          state = 2;
        } else {
          sum += x[r] & VAL;
          ++used;
          if (st == 2) state = 1;
        }
      }
    }
    uint32_t tot = sum;
    int adv = used, fin = state == 1;
    if (G > 1) {
      tot = 0;
      adv = 0;
      fin = 0;
      bool stop = false;
#pragma unroll
      for (int qq = 0; qq < G; ++qq) {
        const uint32_t s_q = __shfl(sum, gl + qq, 64);
        const int u_q = __shfl(used, gl + qq, 64);
        const int st_q = __shfl(state, gl + qq, 64);
        if (!stop) {
          tot += s_q;
          adv += u_q;
          if (st_q != 0) {
            stop = true;
            fin = st_q == 1;
          }
        }
      }
    }
    excl += tot;
    if (fin) break;
    j -= adv;
    if (adv == 0) {
      if (++spins > LB_SPIN_LIMIT) {
        atomicOr(err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (q == 0) st_u32(my, PFX | (excl + run));
  return excl;
}

template <typename K, int NTB, int IPT, int LBR>
__global__ __launch_bounds__(NTB) void k_sp_pass2(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                  K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                  const uint64_t* __restrict__ d_n, int shift,
                                                  const uint32_t* __restrict__ ghist, uint32_t* __restrict__ desc,
                                                  uint32_t* __restrict__ err, uint64_t* __restrict__ stamp) {
  constexpr int NW = NTB / 64, G = NTB / RS_BINS, WT = 64 * IPT, TILE = NTB * IPT;
  static_assert(G == 1 || G == 2 || G == 4, "threads per digit");
  __shared__ uint16_t s_cnt[IPT][NW][RS_BINS];
  __shared__ uint32_t s_base[RS_BINS];
  __shared__ uint32_t s_dbase[RS_BINS];
  __shared__ uint32_t s_wsum[4];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  if (blockIdx.x >= ntiles) return;
  if (t < RS_BINS) {  // digit bases: exclusive scan of the global histogram
    const uint32_t h = hist_total(ghist, t);
    uint32_t inc = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wsum[wv] = inc;
    s_dbase[t] = inc - h;
  }
  __syncthreads();
  if (t < RS_BINS)
    for (int w = 0; w < wv; ++w) s_dbase[t] += s_wsum[w];
  const uint64_t lt = lane_mask_lt();
  const int dd_d = t / G, dd_q = t % G;  // digit group of this thread
  constexpr int WPQ = NW / G;            // waves summed by each thread of a digit group
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == blockIdx.x;
    sp_stamp(stamp, first, 0);
    {
      uint32_t* z = (uint32_t*)&s_cnt[0][0][0];
      for (int i = t; i < IPT * NW * RS_BINS / 2; i += NTB) z[i] = 0;
    }
    __syncthreads();
    const uint64_t b0 = tile * TILE + (uint64_t)wv * WT + lane;
    K k[IPT];
    uint32_t v[IPT], dg[IPT], rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint64_t j = b0 + (uint64_t)i * 64;
      k[i] = j < n ? kin[j] : (K)0;
      v[i] = j < n ? vin[j] : 0u;
    }
    if (stamp) {
      uint64_t z = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) z |= (uint64_t)k[i] ^ v[i];
      if (z == 0x5a5a5a5a5a5aull) stamp[0] = z;
      sp_stamp(stamp, first, 1);
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const bool ok = b0 + (uint64_t)i * 64 < n;
      const uint32_t d = (uint32_t)(k[i] >> shift) & 0xffu;
      dg[i] = d;
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint64_t bb = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bb : ~bb;
      }
      rk[i] = (uint32_t)__popcll(peers & lt);
      if (ok && (peers & lt) == 0) s_cnt[i][wv][d] = (uint16_t)__popcll(peers);
    }
    __syncthreads();
    sp_stamp(stamp, first, 2);
    // digit group (d, q): waves [q WPQ, (q+1) WPQ) in tile order (wave-major, substep-minor)
    uint32_t loc = 0;
#pragma unroll
    for (int w = 0; w < WPQ; ++w)
#pragma unroll
      for (int i = 0; i < IPT; ++i) loc += s_cnt[i][dd_q * WPQ + w][dd_d];
    uint32_t before = 0, run = loc;
    if (G > 1) {
      const int gl = lane & ~(G - 1);
      run = 0;
#pragma unroll
      for (int qq = 0; qq < G; ++qq) {
        const uint32_t x = __shfl(loc, gl + qq, 64);
        before += qq < dd_q ? x : 0u;
        run += x;
      }
    }
    uint32_t acc = before;
#pragma unroll
    for (int w = 0; w < WPQ; ++w)
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const uint32_t c = s_cnt[i][dd_q * WPQ + w][dd_d];
        s_cnt[i][dd_q * WPQ + w][dd_d] = (uint16_t)acc;
        acc += c;
      }
    const uint32_t excl = osg_lookback<G, LBR>(desc, tile, dd_d, dd_q, run, err);
    if (dd_q == 0) s_base[dd_d] = s_dbase[dd_d] + excl;
    __syncthreads();
    sp_stamp(stamp, first, 3);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      if (b0 + (uint64_t)i * 64 < n) {
        const uint64_t pos = (uint64_t)s_base[dg[i]] + s_cnt[i][wv][dg[i]] + rk[i];
        kout[pos] = k[i];
        vout[pos] = v[i];
      }
    }
    __syncthreads();
    sp_stamp(stamp, first, 4);
  }
}

// ---------------------------------------------------------------- onesweep pass, 1024-thread tiles
// Same contract as k_sp_pass.  A tile is 16 waves x IPT substeps x 64 keys, so a
// tile needs few serial substeps per wave and a small grid covers the keys;
// per-(substep, wave, digit) counts are u16 in LDS, written by the digit
// group's leader lane without read-modify-write.  Four threads serve each
// digit: they prefix-sum the counts and read 64 predecessors per look-back
// round trip between them.
constexpr int OSB_NT = 1024;
constexpr int OSB_NW = OSB_NT / 64;

__device__ __forceinline__ uint32_t osb_lookback(uint32_t* desc, uint64_t tile, int d, int q, uint32_t run,
                                                 uint32_t* err) {
  constexpr uint32_t AGG = 1u << 30, PFX = 2u << 30, VAL = AGG - 1;
  constexpr int R = 16;
  uint32_t* my = desc + tile * RS_BINS + d;
  if (tile == 0) {
    if (q == 0) st_u32(my, PFX | run);
    return 0;
  }
  if (q == 0) st_u32(my, AGG | run);
  const int gl = lane_id() & ~3;
  uint32_t excl = 0, spins = 0;
  int64_t j = (int64_t)tile - 1;
  while (true) {
    uint32_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t jj = j - (int64_t)(q * R + r);
      x[r] = jj >= 0 ? ld_u32(desc + (uint64_t)jj * RS_BINS + d) : PFX;
    }
    uint32_t sum = 0;
    int used = 0, state = 0;  // state: 0 open, 1 found a prefix, 2 blocked
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (state == 0) {
        const uint32_t st = x[r] >> 30;
        if (st == 0) {
          state = 2;
        } else {
          sum += x[r] & VAL;
          ++used;
          if (st == 2) state = 1;
        }
      }
    }
    uint32_t tot = 0;
    int adv = 0, fin = 0;
    bool stop = false;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const uint32_t s_q = __shfl(sum, gl + qq, 64);
      const int u_q = __shfl(used, gl + qq, 64);
      const int st_q = __shfl(state, gl + qq, 64);
      if (!stop) {
        tot += s_q;
        adv += u_q;
        if (st_q != 0) {
          stop = true;
          fin = st_q == 1;
        }
      }
    }
    excl += tot;
    if (fin) break;
    j -= adv;
    if (adv == 0) {
      if (++spins > LB_SPIN_LIMIT) {
        atomicOr(err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (q == 0) st_u32(my, PFX | (excl + run));
  return excl;
}

template <typename K, int IPT>
__global__ __launch_bounds__(OSB_NT) void k_sp_passb(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                     K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                     const uint64_t* __restrict__ d_n, int shift,
                                                     const uint32_t* __restrict__ ghist, uint32_t* __restrict__ desc,
                                                     uint32_t* __restrict__ err, uint64_t* __restrict__ stamp) {
  constexpr int WT = 64 * IPT, TILE = OSB_NT * IPT;
  __shared__ uint16_t s_cnt[IPT][OSB_NW][RS_BINS];
  __shared__ uint32_t s_base[RS_BINS];
  __shared__ uint32_t s_dbase[RS_BINS];
  __shared__ uint32_t s_wsum[4];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  if (blockIdx.x >= ntiles) return;
  // digit bases: exclusive scan of the global histogram (waves 0-3)
  if (t < RS_BINS) {
    const uint32_t h = hist_total(ghist, t);
    uint32_t inc = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wsum[wv] = inc;
    s_dbase[t] = inc - h;
  }
  __syncthreads();
  if (t < RS_BINS)
    for (int w = 0; w < wv; ++w) s_dbase[t] += s_wsum[w];
  const uint64_t lt = lane_mask_lt();
  const int dg_d = t >> 2, dg_q = t & 3;  // digit group of this thread
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == blockIdx.x;
    sp_stamp(stamp, first, 0);
    {
      uint32_t* z = (uint32_t*)&s_cnt[0][0][0];
      for (int i = t; i < IPT * OSB_NW * RS_BINS / 2; i += OSB_NT) z[i] = 0;
    }
    __syncthreads();
    const uint64_t b0 = tile * TILE + (uint64_t)wv * WT + lane;
    K k[IPT];
    uint32_t v[IPT], dg[IPT], rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint64_t j = b0 + (uint64_t)i * 64;
      k[i] = j < n ? kin[j] : (K)0;
      v[i] = j < n ? vin[j] : 0u;
    }
    if (stamp) {
      uint64_t z = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) z |= (uint64_t)k[i] ^ v[i];
      if (z == 0x5a5a5a5a5a5aull) stamp[0] = z;
      sp_stamp(stamp, first, 1);
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const bool ok = b0 + (uint64_t)i * 64 < n;
      const uint32_t d = (uint32_t)(k[i] >> shift) & 0xffu;
      dg[i] = d;
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint64_t bb = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bb : ~bb;
      }
      rk[i] = (uint32_t)__popcll(peers & lt);
      if (ok && (peers & lt) == 0) s_cnt[i][wv][d] = (uint16_t)__popcll(peers);
    }
    __syncthreads();
    sp_stamp(stamp, first, 2);
    // digit group (d, q): waves 4q..4q+3 in tile order (wave-major, substep-minor)
    uint32_t loc = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int i = 0; i < IPT; ++i) loc += s_cnt[i][dg_q * 4 + w][dg_d];
    const int gl = lane & ~3;
    uint32_t before = 0, run = 0;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const uint32_t x = __shfl(loc, gl + qq, 64);
      before += qq < dg_q ? x : 0u;
      run += x;
    }
    uint32_t acc = before;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const uint32_t c = s_cnt[i][dg_q * 4 + w][dg_d];
        s_cnt[i][dg_q * 4 + w][dg_d] = (uint16_t)acc;
        acc += c;
      }
    const uint32_t excl = osb_lookback(desc, tile, dg_d, dg_q, run, err);
    if (dg_q == 0) s_base[dg_d] = s_dbase[dg_d] + excl;
    __syncthreads();
    sp_stamp(stamp, first, 3);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      if (b0 + (uint64_t)i * 64 < n) {
        const uint64_t pos = (uint64_t)s_base[dg[i]] + s_cnt[i][wv][dg[i]] + rk[i];
        kout[pos] = k[i];
        vout[pos] = v[i];
      }
    }
    __syncthreads();
    sp_stamp(stamp, first, 4);
  }
}

// ---------------------------------------------------------------- bucket kernel
// After one stable MSD pass on the top 8 key bits the records form 256
// buckets (ascending u), each in emission order (ascending v).  One 1024-thread
// workgroup per bucket: bitonic sort of (key, position) in LDS -- position
// breaks ties, so runs keep ascending v -- then one thread per position scores
// the run starting there (first-order exclusion, metric, minScore filter) and
// the bucket's candidates are compacted in (u, w) order behind the preceding
// buckets (look-back over bucket ids).  A bucket above BK_CAP raises F_TOOBIG
// (the host then takes the LSD path).
constexpr int BK_NT = 1024;
constexpr int BK_NW = BK_NT / 64;
constexpr int BK_CAP = 4096;
constexpr int BK_PER = BK_CAP / BK_NT;

// SORT_ONLY: stop after the bucket sort and write it back in place -- sorted
// keys to rkey, for every run start its length to rlen (0 elsewhere), and
// (CUSTOM) the values in sorted order to vsorted -- for k_sp_runs, which scores
// the runs with the whole chip instead of one workgroup per bucket (a hub's
// bucket would otherwise keep one CU busy long after the others).
template <bool CUSTOM, bool SORT_ONLY = false>
__global__ __launch_bounds__(BK_NT) void k_sp_bucket(GraphView g, int metric, float min_score, uint64_t ua,
                                                     int wbits, const uint64_t* __restrict__ rkey,
                                                     const uint32_t* __restrict__ rval,
                                                     const uint32_t* __restrict__ bhist /*256*/,
                                                     uint32_t* __restrict__ cu, uint32_t* __restrict__ cw,
                                                     float* __restrict__ cs, uint32_t* __restrict__ okey,
                                                     uint32_t* __restrict__ oval, uint64_t* __restrict__ desc,
                                                     uint64_t* __restrict__ ctr, int lbits, uint64_t kmax,
                                                     uint32_t* __restrict__ ohist /*4 x 256*/,
                                                     uint64_t* __restrict__ stamp, uint64_t* __restrict__ skey = nullptr,
                                                     uint32_t* __restrict__ rlen = nullptr,
                                                     uint32_t* __restrict__ vsorted = nullptr) {
  __shared__ uint64_t s_k2[2][BK_CAP];
  __shared__ uint32_t s_oh[1][RS_BINS];
  __shared__ uint16_t s_p2[2][BK_CAP];
  __shared__ uint16_t s_cnt[BK_PER][BK_NW][RS_BINS];
  __shared__ uint32_t s_dig[RS_BINS];
  __shared__ uint16_t s_rs[BK_CAP + 1];  // start position of each (u, w) run
  __shared__ uint32_t s_wsum[BK_NW];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_start, s_bcnt;
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint32_t b = blockIdx.x;
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  const uint64_t n = ctr[C_WSORT];
  sp_stamp(stamp, true, 0);
  // bucket bounds: exclusive prefix of the digit histogram (threads 0-255 hold the bins)
  {
    const uint32_t h = (n && t < RS_BINS) ? hist_total(bhist, t) : 0u;
    uint32_t inc = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = inc - h;
    for (int w = 0; w < wv; ++w) pre += s_wsum[w];
    if (t == (int)b) {
      s_start = pre;
      s_bcnt = h;
    }
    __syncthreads();
  }
  const uint32_t start = s_start, c = s_bcnt;
  sp_stamp(stamp, true, 1);
  if (t < RS_BINS) s_oh[0][t] = 0;
  const bool toobig = c > (uint32_t)BK_CAP;
  if (toobig && t == 0) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_TOOBIG);
  const uint32_t m = toobig ? 0u : c;
  for (uint32_t i = t; i < m; i += BK_NT) {
    s_k2[0][i] = rkey[start + i];
    s_p2[0][i] = (uint16_t)i;
  }
  __syncthreads();
  sp_stamp(stamp, true, 2);
  // stable LSD radix sort in LDS by the key bits below the bucket digit;
  // items striped i = r * 1024 + t, ranked in (r, wave, lane) = index order
  const uint64_t lt = lane_mask_lt();
  const int rmax = (int)((m + BK_NT - 1) / BK_NT);
  int cur = 0;
  for (int sh = 0; sh < lbits; sh += 8) {
    {
      uint32_t* z = (uint32_t*)&s_cnt[0][0][0];
      for (int i = t; i < BK_PER * BK_NW * RS_BINS / 2; i += BK_NT) z[i] = 0;
    }
    __syncthreads();
    uint64_t kk[BK_PER];
    uint16_t pp[BK_PER];
    uint32_t dd[BK_PER], rk[BK_PER];
#pragma unroll
    for (int r = 0; r < BK_PER; ++r) {
      if (r < rmax) {
        const uint32_t i = (uint32_t)r * BK_NT + t;
        const bool ok = i < m;
        kk[r] = ok ? s_k2[cur][i] : 0ull;
        pp[r] = ok ? s_p2[cur][i] : (uint16_t)0;
        const uint32_t d = (uint32_t)(kk[r] >> sh) & 0xffu;
        dd[r] = d;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int bt = 0; bt < 8; ++bt) {
          const uint64_t bb = __ballot((d >> bt) & 1u);
          peers &= ((d >> bt) & 1u) ? bb : ~bb;
        }
        rk[r] = (uint32_t)__popcll(peers & lt);
        if (ok && (peers & lt) == 0) s_cnt[r][wv][d] = (uint16_t)__popcll(peers);
      }
    }
    __syncthreads();
    // digit t: exclusive prefix over (r, wave); then the digit bases
    uint32_t tot = 0;
    if (t < RS_BINS) {
      for (int r = 0; r < rmax; ++r)
        for (int w = 0; w < BK_NW; ++w) {
          const uint32_t c2 = s_cnt[r][w][t];
          s_cnt[r][w][t] = (uint16_t)tot;
          tot += c2;
        }
      uint32_t inc = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      if (lane == 63) s_wsum[wv] = inc;
      s_dig[t] = inc - tot;
    }
    __syncthreads();
    if (t < RS_BINS)
      for (int w = 0; w < wv; ++w) s_dig[t] += s_wsum[w];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < BK_PER; ++r) {
      if (r < rmax && (uint32_t)r * BK_NT + t < m) {
        const uint32_t pos = s_dig[dd[r]] + s_cnt[r][wv][dd[r]] + rk[r];
        s_k2[cur ^ 1][pos] = kk[r];
        s_p2[cur ^ 1][pos] = pp[r];
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  const uint64_t* s_key = s_k2[cur];
  const uint16_t* s_pos = s_p2[cur];
  float* s_sc = (float*)s_k2[cur ^ 1];                  // the free buffer holds scores ...
  uint32_t* s_flag = (uint32_t*)s_k2[cur ^ 1] + BK_CAP;  // ... and flags
  sp_stamp(stamp, true, 3);
  // (u, w) runs: block scan of the run starts (positions blocked 4 per thread)
  // gives every run its start, so no thread walks a run position by position
  // (two hubs can share long runs).
  uint32_t R;
  {
    uint32_t sf[BK_PER], ns = 0;
#pragma unroll
    for (int r = 0; r < BK_PER; ++r) {
      const uint32_t p = (uint32_t)t * BK_PER + r;
      sf[r] = (p < m && (p == 0 || s_key[p - 1] != s_key[p])) ? 1u : 0u;
      ns += sf[r];
    }
    uint32_t inc = ns;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wsum[wv] = inc;
    __syncthreads();
    uint32_t id = inc - ns;
    R = 0;
    for (int w = 0; w < BK_NW; ++w) {
      const uint32_t x = s_wsum[w];
      id += w < wv ? x : 0u;
      R += x;
    }
#pragma unroll
    for (int r = 0; r < BK_PER; ++r)
      if (sf[r]) s_rs[id++] = (uint16_t)((uint32_t)t * BK_PER + r);
    if (t == 0) s_rs[R] = (uint16_t)m;
    __syncthreads();
  }
  if (SORT_ONLY) {
    if (toobig)  // no runs from this bucket (the host reruns with the LSD sort)
      for (uint32_t i = t; i < c; i += BK_NT) rlen[start + i] = 0u;
    for (uint32_t i = t; i < m; i += BK_NT) {
      skey[start + i] = s_key[i];
      rlen[start + i] = 0u;
      if (CUSTOM) vsorted[start + i] = rval[start + s_pos[i]];
    }
    __syncthreads();
    for (uint32_t r = t; r < R; r += BK_NT) rlen[start + s_rs[r]] = (uint32_t)s_rs[r + 1] - s_rs[r];
    sp_stamp(stamp, true, 4);
    return;
  }
  // score the runs (striped r = t + 1024 j); a thread's runs issue their
  // independent loads and the steps of their membership searches side by side
  const uint64_t wmask = (1ull << wbits) - 1;
  uint32_t ru[BK_PER], rw[BK_PER], rc[BK_PER], lo[BK_PER], hi[BK_PER], du[BK_PER], dw[BK_PER], tg[BK_PER];
  uint32_t ln[BK_PER];
  const uint32_t* rl[BK_PER];
  float racc[BK_PER];
  bool has[BK_PER];
#pragma unroll
  for (int j = 0; j < BK_PER; ++j) {
    const uint32_t r = (uint32_t)t + (uint32_t)j * BK_NT;
    has[j] = r < R;
    if (has[j]) {
      const uint32_t p = s_rs[r], cnt = (uint32_t)s_rs[r + 1] - p;
      const uint64_t k = s_key[p];
      float acc = 0.0f;
      if (CUSTOM)  // the reference's order: ascending v (= ascending position)
        for (uint32_t q = p; q < p + cnt; ++q) acc = (float)((double)acc + g.ctab[g.deg[rval[start + s_pos[q]]]]);
      ru[j] = (uint32_t)(ua + (k >> wbits));
      rw[j] = (uint32_t)(k & wmask);
      rc[j] = cnt;
      racc[j] = acc;
    }
  }
  // First-order exclusion: w in N(u) <=> u in I(w) (the transposed lists, the
  // same arrays when the graph is symmetric); search the shorter sorted list, so
  // a hub u's candidates are checked against their small in-lists.
  const bool sym = g.toff == g.off;
#pragma unroll
  for (int j = 0; j < BK_PER; ++j) {
    if (has[j]) {
      const uint64_t ou = g.off[ru[j]], ou1 = g.off[ru[j] + 1];
      const uint64_t tw = g.toff[rw[j]], tw1 = g.toff[rw[j] + 1];
      du[j] = (uint32_t)(ou1 - ou);
      const uint32_t iw = (uint32_t)(tw1 - tw);
      dw[j] = CUSTOM ? 0u : (sym ? iw : g.deg[rw[j]]);
      const bool via_w = iw < du[j];
      rl[j] = via_w ? g.tkeys + tw : g.keys + ou;
      tg[j] = via_w ? ru[j] : rw[j];
      ln[j] = via_w ? iw : du[j];
    } else {
      rl[j] = g.keys;
      tg[j] = 0;
      ln[j] = 0;
    }
    lo[j] = 0;
    hi[j] = ln[j];
  }
  bool more = true;
  while (more) {  // lower bounds, in lockstep
    more = false;
    uint32_t mid[BK_PER], av[BK_PER];
#pragma unroll
    for (int j = 0; j < BK_PER; ++j) {
      mid[j] = (lo[j] + hi[j]) >> 1;
      av[j] = lo[j] < hi[j] ? rl[j][mid[j]] : 0u;
    }
#pragma unroll
    for (int j = 0; j < BK_PER; ++j) {
      if (lo[j] < hi[j]) {
        if (av[j] < tg[j]) lo[j] = mid[j] + 1;
        else hi[j] = mid[j];
        more |= lo[j] < hi[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < BK_PER; ++j) {
    if (has[j]) {
      const uint32_t r = (uint32_t)t + (uint32_t)j * BK_NT;
      const bool excl = lo[j] < ln[j] && rl[j][lo[j]] == tg[j];
      float sc;
      if (CUSTOM) sc = excl ? 0.0f : racc[j];
      else sc = score_basic(metric, excl ? 0u : rc[j], du[j], dw[j]);
      s_sc[r] = sc;
      s_flag[r] = !(sc <= min_score) ? 1u : 0u;  // NaN passes
    }
  }
  __syncthreads();
  sp_stamp(stamp, true, 4);
  // blocked scan of the run flags: thread t owns runs [4t, 4t+4)
  uint32_t f[BK_PER], tsum = 0;
#pragma unroll
  for (int r = 0; r < BK_PER; ++r) {
    const uint32_t q = (uint32_t)t * BK_PER + r;
    f[r] = q < R ? s_flag[q] : 0u;
    tsum += f[r];
  }
  uint32_t inc = tsum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_wsum[wv] = inc;
  __syncthreads();
  uint32_t pre = inc - tsum, agg = 0;
  for (int w = 0; w < BK_NW; ++w) {
    const uint32_t x = s_wsum[w];
    pre += w < wv ? x : 0u;
    agg += x;
  }
  if (wv == 0) {
    const uint64_t e = lb_lookback_r<4>(desc, b, agg, err);
    if (lane == 0) {
      s_excl = e;
      if (b == gridDim.x - 1) {
        ctr[C_C] = e + agg;
        ctr[C_OUT_N] = std::min<uint64_t>(e + agg, kmax);
      }
    }
  }
  __syncthreads();
  sp_stamp(stamp, true, 5);
  uint64_t o = s_excl + pre;
  uint32_t nnan = 0;
#pragma unroll
  for (int r = 0; r < BK_PER; ++r) {
    if (f[r]) {
      const uint32_t q = (uint32_t)t * BK_PER + r;
      const uint64_t k = s_key[s_rs[q]];
      const float sc = s_sc[q];
      cu[o] = (uint32_t)(ua + (k >> wbits));
      cw[o] = (uint32_t)(k & wmask);
      cs[o] = sc;
      const uint32_t ok = ~score_key(sc);
      okey[o] = ok;
      oval[o] = (uint32_t)o;
      atomicAdd(&s_oh[0][ok & 0xffu], 1u);  // digit 0 only: the first ordering pass counts the rest
      nnan += sc != sc;
      ++o;
    }
  }
  if (nnan) atomicAdd((unsigned long long*)&ctr[C_NAN], (unsigned long long)nnan);
  __syncthreads();
  if (t < RS_BINS) {
    const uint32_t hc = s_oh[0][t];
    if (hc) atomicAdd(&hist_copy(ohist)[t], hc);
  }
  sp_stamp(stamp, true, 6);
}

// ---------------------------------------------------------------- onesweep pass, 512-thread tiles
// Same contract as k_sp_pass (running per-wave digit counters), with 8 waves of
// IPT keys each: a tile of 4096 keys takes half the serial ranking steps per
// wave, and two threads per digit read 2 x LBR predecessors per look-back
// round trip (one round trip for up to 64 tiles with LBR = 32).
template <typename K, int IPT, int LBR>
__global__ __launch_bounds__(512) void k_sp_pass3(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                  K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                  const uint64_t* __restrict__ d_n, int shift,
                                                  const uint32_t* __restrict__ ghist, uint32_t* __restrict__ desc,
                                                  uint32_t* __restrict__ err, uint64_t* __restrict__ stamp,
                                                  uint32_t* __restrict__ nhist) {
  constexpr int NTB = 512, NW = 8, WT = 64 * IPT, TILE = NTB * IPT;
  __shared__ uint32_t s_wcnt[NW][RS_BINS];
  __shared__ uint32_t s_base[RS_BINS];
  __shared__ uint32_t s_dbase[RS_BINS];
  __shared__ uint32_t s_wsum[4];
  __shared__ uint32_t s_nh[3][RS_BINS];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  if (blockIdx.x >= ntiles) return;
  if (t < RS_BINS) {
    const uint32_t h = hist_total(ghist, t);
    uint32_t inc = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wsum[wv] = inc;
    s_dbase[t] = inc - h;
  }
  if (nhist)
    for (int i = t; i < 3 * RS_BINS; i += NTB) (&s_nh[0][0])[i] = 0;
  __syncthreads();
  if (t < RS_BINS)
    for (int w = 0; w < wv; ++w) s_dbase[t] += s_wsum[w];
  const uint64_t lt = lane_mask_lt();
  const int dd_d = t >> 1, dd_q = t & 1;  // two threads per digit
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == blockIdx.x;
    sp_stamp(stamp, first, 0);
    for (int i = t; i < NW * RS_BINS; i += NTB) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t b0 = tile * TILE + (uint64_t)wv * WT + lane;
    K k[IPT];
    uint32_t v[IPT], dg[IPT], rk[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint64_t j = b0 + (uint64_t)i * 64;
      k[i] = j < n ? kin[j] : (K)0;
      v[i] = j < n ? vin[j] : 0u;
    }
    if (stamp) {
      uint64_t z = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) z |= (uint64_t)k[i] ^ v[i];
      if (z == 0x5a5a5a5a5a5aull) stamp[0] = z;
      sp_stamp(stamp, first, 1);
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
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
    sp_stamp(stamp, first, 2);
    // digit pair (d, q): waves 4q..4q+3, combined by one shuffle
    uint32_t loc = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) loc += s_wcnt[dd_q * 4 + w][dd_d];
    const uint32_t other = __shfl_xor(loc, 1, 64);
    const uint32_t run = loc + other;
    uint32_t acc = dd_q ? other : 0u;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t c = s_wcnt[dd_q * 4 + w][dd_d];
      s_wcnt[dd_q * 4 + w][dd_d] = acc;
      acc += c;
    }
    const uint32_t excl = osg_lookback<2, LBR>(desc, tile, dd_d, dd_q, run, err);
    if (dd_q == 0) s_base[dd_d] = s_dbase[dd_d] + excl;
    __syncthreads();
    sp_stamp(stamp, first, 3);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      if (b0 + (uint64_t)i * 64 < n) {
        const uint64_t pos = (uint64_t)s_base[dg[i]] + s_wcnt[wv][dg[i]] + rk[i];
        kout[pos] = k[i];
        vout[pos] = v[i];
        if (nhist) {
#pragma unroll
          for (int dd = 0; dd < 3; ++dd) atomicAdd(&s_nh[dd][(uint32_t)(k[i] >> (8 * dd + 8)) & 0xffu], 1u);
        }
      }
    }
    __syncthreads();
    sp_stamp(stamp, first, 4);
  }
  if (nhist) {
    uint32_t* hc = hist_copy(nhist);
    for (int i = t; i < 3 * RS_BINS; i += NTB) {
      const uint32_t c = s_nh[i / RS_BINS][i % RS_BINS];
      if (c) atomicAdd(&hc[i], c);
    }
  }
}

// ---------------------------------------------------------------- group sort
// After P stable MSD passes the records are grouped by their top 8P key bits
// ("fine buckets", ascending).  Workgroup b takes the fine buckets that start
// in records [b*GR_T, (b+1)*GR_T): its range is cut at fine-bucket boundaries
// found by scanning the keys, so neighbouring workgroups agree and the ranges
// partition the records.  It sorts the range in LDS by the key bits that vary
// inside it (stable LSD, ballot multisplit), then writes back in place the
// sorted keys, the run lengths at run starts (0 elsewhere) and, for the
// Adamic-Adar / Resource-Allocation sums, the values in sorted order.  A range
// above BK_CAP records raises F_TOOBIG (the host then reruns with more MSD
// passes or the full LSD sort).
constexpr uint32_t GR_T = 1024;

template <bool CUSTOM>
__global__ __launch_bounds__(BK_NT) void k_sp_group(const uint64_t* __restrict__ rkey_in,
                                                    const uint32_t* __restrict__ rval, int fshift,
                                                    uint64_t* __restrict__ skey, uint32_t* __restrict__ rlen,
                                                    uint32_t* __restrict__ vsorted, uint64_t* __restrict__ ctr,
                                                    uint64_t* __restrict__ stamp) {
  __shared__ uint64_t s_k2[2][BK_CAP];
  __shared__ uint16_t s_p2[2][BK_CAP];
  __shared__ uint16_t s_cnt[BK_PER][BK_NW][RS_BINS];
  __shared__ uint32_t s_dig[RS_BINS];
  __shared__ uint16_t s_rs[BK_CAP + 1];
  __shared__ uint32_t s_wsum[BK_NW];
  __shared__ uint64_t s_bnd[2];
  __shared__ uint64_t s_or[BK_NW], s_and[BK_NW];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = ctr[C_WSORT];
  const uint64_t x0 = (uint64_t)blockIdx.x * GR_T;
  if (x0 >= n) return;
  sp_stamp(stamp, true, 0);
  // range bounds: the first fine-bucket boundary at or after x0 and x1
  for (int e = 0; e < 2; ++e) {
    const uint64_t x = std::min<uint64_t>(x0 + (uint64_t)e * GR_T, n);
    if (t == 0) s_bnd[e] = ~0ull;
    __syncthreads();
    if (x == 0 || x == n) {
      if (t == 0) s_bnd[e] = x;
    } else {
      for (uint64_t c0 = x; c0 < n && c0 < x + BK_CAP + 1; c0 += BK_NT) {
        const uint64_t i = c0 + t;
        const bool bd = i < n && (rkey_in[i] >> fshift) != (rkey_in[i - 1] >> fshift);
        const bool end = i == n;
        if (bd || end) atomicMin((unsigned long long*)&s_bnd[e], (unsigned long long)i);
        __syncthreads();
        if (s_bnd[e] != ~0ull) break;
        __syncthreads();
      }
      if (t == 0 && s_bnd[e] == ~0ull) s_bnd[e] = std::min<uint64_t>(n, x + BK_CAP + 1);  // too long: flagged below
    }
    __syncthreads();
  }
  const uint64_t start = s_bnd[0], stop = s_bnd[1];
  if (stop <= start) return;  // the range begins in a neighbour's fine bucket
  const uint64_t c = stop - start;
  if (c > BK_CAP) {
    if (t == 0) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_TOOBIG);
    for (uint64_t i = start + t; i < stop; i += BK_NT) rlen[i] = 0u;
    return;
  }
  const uint32_t m = (uint32_t)c;
  uint64_t ko = 0, ka = ~0ull;
  for (uint32_t i = t; i < m; i += BK_NT) {
    const uint64_t k = rkey_in[start + i];
    s_k2[0][i] = k;
    s_p2[0][i] = (uint16_t)i;
    ko |= k;
    ka &= k;
  }
  // the bits that vary inside the range decide the number of LDS passes
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ko |= __shfl_xor(ko, o, 64);
    ka &= __shfl_xor(ka, o, 64);
  }
  if (lane == 0) {
    s_or[wv] = ko;
    s_and[wv] = ka;
  }
  __syncthreads();
  // bits that differ anywhere in the range: (OR of all keys) ^ (AND of all keys)
  // -- per-wave OR ^ AND would miss bits constant inside each wave but different
  // between waves (consecutive fine buckets split across waves)
  uint64_t all_or = 0, all_and = ~0ull;
  for (int w = 0; w < BK_NW; ++w) {
    all_or |= s_or[w];
    all_and &= s_and[w];
  }
  const uint64_t diff = m ? all_or ^ all_and : 0;
  const int lbits = diff ? 64 - __clzll((long long)diff) : 0;
  sp_stamp(stamp, true, 1);
  const uint64_t lt = lane_mask_lt();
  const int rmax = (int)((m + BK_NT - 1) / BK_NT);
  int cur = 0;
  for (int sh = 0; sh < lbits; sh += 8) {
    {
      uint32_t* z = (uint32_t*)&s_cnt[0][0][0];
      for (int i = t; i < BK_PER * BK_NW * RS_BINS / 2; i += BK_NT) z[i] = 0;
    }
    __syncthreads();
    uint64_t kk[BK_PER];
    uint16_t pp[BK_PER];
    uint32_t dd[BK_PER], rk[BK_PER];
#pragma unroll
    for (int r = 0; r < BK_PER; ++r) {
      if (r < rmax) {
        const uint32_t i = (uint32_t)r * BK_NT + t;
        const bool ok = i < m;
        kk[r] = ok ? s_k2[cur][i] : 0ull;
        pp[r] = ok ? s_p2[cur][i] : (uint16_t)0;
        const uint32_t d = (uint32_t)(kk[r] >> sh) & 0xffu;
        dd[r] = d;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int bt = 0; bt < 8; ++bt) {
          const uint64_t bb = __ballot((d >> bt) & 1u);
          peers &= ((d >> bt) & 1u) ? bb : ~bb;
        }
        rk[r] = (uint32_t)__popcll(peers & lt);
        if (ok && (peers & lt) == 0) s_cnt[r][wv][d] = (uint16_t)__popcll(peers);
      }
    }
    __syncthreads();
    uint32_t tot = 0;
    if (t < RS_BINS) {
      for (int r = 0; r < rmax; ++r)
        for (int w = 0; w < BK_NW; ++w) {
          const uint32_t c2 = s_cnt[r][w][t];
          s_cnt[r][w][t] = (uint16_t)tot;
          tot += c2;
        }
      uint32_t inc = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      if (lane == 63) s_wsum[wv] = inc;
      s_dig[t] = inc - tot;
    }
    __syncthreads();
    if (t < RS_BINS)
      for (int w = 0; w < wv; ++w) s_dig[t] += s_wsum[w];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < BK_PER; ++r) {
      if (r < rmax && (uint32_t)r * BK_NT + t < m) {
        const uint32_t pos = s_dig[dd[r]] + s_cnt[r][wv][dd[r]] + rk[r];
        s_k2[cur ^ 1][pos] = kk[r];
        s_p2[cur ^ 1][pos] = pp[r];
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  const uint64_t* s_key = s_k2[cur];
  const uint16_t* s_pos = s_p2[cur];
  sp_stamp(stamp, true, 2);
  // run starts (blocked 4 per thread) -> run ids -> start positions
  uint32_t R;
  {
    uint32_t sf[BK_PER], ns = 0;
#pragma unroll
    for (int r = 0; r < BK_PER; ++r) {
      const uint32_t p = (uint32_t)t * BK_PER + r;
      sf[r] = (p < m && (p == 0 || s_key[p - 1] != s_key[p])) ? 1u : 0u;
      ns += sf[r];
    }
    uint32_t inc = ns;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wsum[wv] = inc;
    __syncthreads();
    uint32_t id = inc - ns;
    R = 0;
    for (int w = 0; w < BK_NW; ++w) {
      const uint32_t x = s_wsum[w];
      id += w < wv ? x : 0u;
      R += x;
    }
#pragma unroll
    for (int r = 0; r < BK_PER; ++r)
      if (sf[r]) s_rs[id++] = (uint16_t)((uint32_t)t * BK_PER + r);
    if (t == 0) s_rs[R] = (uint16_t)m;
    __syncthreads();
  }
  for (uint32_t i = t; i < m; i += BK_NT) {
    skey[start + i] = s_key[i];
    rlen[start + i] = 0u;
    if (CUSTOM) vsorted[start + i] = rval[start + s_pos[i]];
  }
  __syncthreads();
  for (uint32_t r = t; r < R; r += BK_NT) rlen[start + s_rs[r]] = (uint32_t)s_rs[r + 1] - s_rs[r];
  sp_stamp(stamp, true, 3);
}

// ---------------------------------------------------------------- balanced run scoring
// Over the bucket-sorted records: thread j of a tile looks at records
// base + r * NT + j; those that start a run (rlen > 0) are scored -- first-order
// exclusion by searching the shorter of N(u) and I(w), the metric, the
// minScore filter -- with the searches of a thread's runs in lockstep.  The
// candidates are compacted in record order ((u, w) order) behind the preceding
// tiles (look-back), and digit 0 of their order keys is counted.
#ifndef NLP_RU_IPT
#define NLP_RU_IPT 4
#endif
constexpr int RU_IPT = NLP_RU_IPT;
constexpr int RU_TILE = NT * RU_IPT;

template <bool CUSTOM>
__global__ __launch_bounds__(NT) void k_sp_runs(GraphView g, int metric, float min_score, uint64_t ua, int wbits,
                                                const uint64_t* __restrict__ skey, const uint32_t* __restrict__ rlen,
                                                const uint32_t* __restrict__ vsorted, uint32_t* __restrict__ cu,
                                                uint32_t* __restrict__ cw, float* __restrict__ cs,
                                                uint32_t* __restrict__ okey, uint32_t* __restrict__ oval,
                                                uint64_t* __restrict__ desc, uint64_t* __restrict__ ctr, uint64_t kmax,
                                                uint32_t* __restrict__ ohist, uint64_t* __restrict__ stamp) {
  __shared__ uint32_t s_f[RU_TILE];
  __shared__ float s_sc[RU_TILE];
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_oh[RS_BINS];
  const int t = threadIdx.x;
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  const uint64_t n = ctr[C_WSORT];
  const uint64_t ntiles = (n + RU_TILE - 1) / RU_TILE;
  if (blockIdx.x >= ntiles) return;
  s_oh[t] = 0;
  const uint64_t wmask = (1ull << wbits) - 1;
  const bool sym = g.toff == g.off;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first = tile == blockIdx.x;
    sp_stamp(stamp, first, 0);
    const uint64_t base = tile * RU_TILE;
    uint32_t ru[RU_IPT], rw[RU_IPT], rc[RU_IPT], lo[RU_IPT], hi[RU_IPT], du[RU_IPT], dw[RU_IPT], tg[RU_IPT],
        ln[RU_IPT];
    const uint32_t* rl[RU_IPT];
    float racc[RU_IPT];
    bool has[RU_IPT];
#pragma unroll
    for (int j = 0; j < RU_IPT; ++j) {
      const uint64_t i = base + (uint64_t)j * NT + t;
      rc[j] = i < n ? rlen[i] : 0u;
      has[j] = rc[j] != 0;
      const uint64_t k = has[j] ? skey[i] : 0ull;
      ru[j] = (uint32_t)(ua + (k >> wbits));
      rw[j] = (uint32_t)(k & wmask);
      float acc = 0.0f;
      if (CUSTOM && has[j])  // the reference's order: ascending v
        for (uint32_t q = 0; q < rc[j]; ++q) acc = (float)((double)acc + g.ctab[g.deg[vsorted[i + q]]]);
      racc[j] = acc;
    }
#pragma unroll
    for (int j = 0; j < RU_IPT; ++j) {
      if (has[j]) {
        const uint64_t ou = g.off[ru[j]], ou1 = g.off[ru[j] + 1];
        const uint64_t tw = g.toff[rw[j]], tw1 = g.toff[rw[j] + 1];
        du[j] = (uint32_t)(ou1 - ou);
        const uint32_t iw = (uint32_t)(tw1 - tw);
        dw[j] = CUSTOM ? 0u : (sym ? iw : g.deg[rw[j]]);
        const bool via_w = iw < du[j];
        rl[j] = via_w ? g.tkeys + tw : g.keys + ou;
        tg[j] = via_w ? ru[j] : rw[j];
        ln[j] = via_w ? iw : du[j];
        if (g.efbits) {  // not in the edge filter: w is not in N(u), no search
          const uint64_t h = edge_slot(ru[j], rw[j], g.efbits);
          if (!((g.efilt[h >> 5] >> (h & 31)) & 1u)) ln[j] = 0;
        }
      } else {
        rl[j] = g.keys;
        tg[j] = 0;
        ln[j] = 0;
        du[j] = dw[j] = 0;
      }
      lo[j] = 0;
      hi[j] = ln[j];
    }
    // lower bounds, in lockstep, 4-way: the lower bound lies in [lo, hi]; each
    // round trip loads the last element of the first three quarters, so a
    // search takes log4 instead of log2 dependent loads
    bool more = true;
    while (more) {
      more = false;
      uint32_t st[RU_IPT], pv[RU_IPT][3];
#pragma unroll
      for (int j = 0; j < RU_IPT; ++j) {
        st[j] = (hi[j] - lo[j] + 3) >> 2;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const uint32_t idx = lo[j] + (uint32_t)(q + 1) * st[j] - 1;
          pv[j][q] = (lo[j] < hi[j] && idx < hi[j]) ? rl[j][idx] : 0xffffffffu;
        }
      }
#pragma unroll
      for (int j = 0; j < RU_IPT; ++j) {
        if (lo[j] < hi[j]) {
          uint32_t c = 0;
#pragma unroll
          for (int q = 0; q < 3; ++q) c += pv[j][q] < tg[j] ? 1u : 0u;  // ascending pivots: a prefix
          const uint32_t p = lo[j] + (c + 1) * st[j] - 1;              // a[p] >= target when valid
          hi[j] = (c < 3 && p < hi[j]) ? p : hi[j];
          lo[j] = lo[j] + c * st[j];
          more |= lo[j] < hi[j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RU_IPT; ++j) {
      uint32_t fl = 0;
      float sc = 0.0f;
      if (has[j]) {
        const bool excl = lo[j] < ln[j] && rl[j][lo[j]] == tg[j];
        if (CUSTOM) sc = excl ? 0.0f : racc[j];
        else sc = score_basic(metric, excl ? 0u : rc[j], du[j], dw[j]);
        fl = !(sc <= min_score) ? 1u : 0u;  // NaN passes
      }
      s_f[j * NT + t] = fl;
      s_sc[j * NT + t] = sc;
    }
    __syncthreads();
    sp_stamp(stamp, first, 1);
    // blocked compaction: thread t owns tile items [4t, 4t+4)
    uint32_t f[RU_IPT];
    uint64_t tsum = 0;
#pragma unroll
    for (int r = 0; r < RU_IPT; ++r) {
      f[r] = s_f[t * RU_IPT + r];
      tsum += f[r];
    }
    uint64_t agg;
    const uint64_t pre = block_excl_scan(tsum, s_red, &agg);
    if (wave_id() == 0) {
      const uint64_t e = lb_lookback_r<4>(desc, tile, agg, err);
      if (lane_id() == 0) {
        s_excl = e;
        if (tile == ntiles - 1) {
          ctr[C_C] = e + agg;
          ctr[C_OUT_N] = std::min<uint64_t>(e + agg, kmax);
        }
      }
    }
    __syncthreads();
    sp_stamp(stamp, first, 2);
    uint64_t o = s_excl + pre;
    uint32_t nnan = 0;
#pragma unroll
    for (int r = 0; r < RU_IPT; ++r) {
      if (f[r]) {
        const uint64_t i = base + (uint64_t)t * RU_IPT + r;
        const uint64_t k = skey[i];
        const float sc = s_sc[t * RU_IPT + r];
        cu[o] = (uint32_t)(ua + (k >> wbits));
        cw[o] = (uint32_t)(k & wmask);
        cs[o] = sc;
        const uint32_t ok = ~score_key(sc);
        okey[o] = ok;
        oval[o] = (uint32_t)o;
        atomicAdd(&s_oh[ok & 0xffu], 1u);
        nnan += sc != sc;
        ++o;
      }
    }
    if (nnan) atomicAdd((unsigned long long*)&ctr[C_NAN], (unsigned long long)nnan);
    __syncthreads();
    sp_stamp(stamp, first, 3);
  }
  const uint32_t hc = s_oh[t];
  if (hc) atomicAdd(&hist_copy(ohist)[t], hc);
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

// The first min(k, C) candidates of the score order -> caller's edges.  Block 0
// also publishes the call's counters into host-mapped memory (hctr): the host
// reads them after the stream's final event, with no copy in between.
__global__ __launch_bounds__(NT) void k_sp_gather(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ cu,
                                                  const uint32_t* __restrict__ cw, const float* __restrict__ cs,
                                                  uint64_t k, EdgeOut* __restrict__ out,
                                                  uint64_t* __restrict__ ctr, uint64_t* __restrict__ hctr) {
  const uint64_t m = std::min<uint64_t>(ctr[C_C], k);
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) ctr[C_OUT_N] = m;
    if (hctr && threadIdx.x < NCTR) hctr[threadIdx.x] = threadIdx.x == C_OUT_N ? m : ctr[threadIdx.x];
    if (hctr) __threadfence_system();
  }
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (uint64_t)gridDim.x * NT) {
    const uint32_t x = idx[i];
    out[i] = EdgeOut{cu[x], cw[x], cs[x]};
  }
}

}  // namespace nlp
