// prims.hpp -- device-wide primitives for the link-prediction pipeline (gfx950).
//
// Everything here is hand-written for CDNA4: 64-lane waves (__ballot is 64-bit,
// __shfl over width 64), 256-thread workgroups (4 waves, one per SIMD), LDS
// histograms and wave-ballot multisplit ranking for a STABLE LSD radix sort
// (stability is what carries the reference's accumulation order through the
// regrouping of wedges).
//
//   scan_excl_u64     exclusive prefix sum (u32 or u64 input -> u64 output)
//   lbs               load-balanced search: slot -> item (upper_bound on offsets)
//   sort_pairs_u64    stable LSD radix sort of (u64 key, u32 value) on chosen bytes
//   sort_u32_desc_idx stable sort of u32 keys descending carrying an index
//   radix_select_kth  k-th largest u32 key + count strictly above it (device-side)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nlp {

constexpr int NT = 256;        // threads per workgroup
constexpr int NWAVE = NT / 64;  // waves per workgroup

#define NLP_HIP(x)                                    \
  do {                                                \
    hipError_t e__ = (x);                             \
    if (e__ != hipSuccess) return e__;                \
  } while (0)

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// Exclusive block scan over NT threads.  `lds` needs NWAVE+1 u64.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t x, uint64_t* lds, uint64_t* total) {
  uint64_t inc = wave_incl_scan(x);
  if (lane_id() == 63) lds[wave_id()] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t run = 0;
    for (int w = 0; w < NWAVE; ++w) { uint64_t t = lds[w]; lds[w] = run; run += t; }
    lds[NWAVE] = run;
  }
  __syncthreads();
  uint64_t r = lds[wave_id()] + inc - x;
  if (total) *total = lds[NWAVE];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------- scan
constexpr int SCAN_IPT = 8;                      // items per thread
constexpr int SCAN_TILE = NT * SCAN_IPT;         // 2048 items per workgroup

template <typename T>
__global__ __launch_bounds__(NT) void k_scan_reduce(const T* __restrict__ in, uint64_t n,
                                                    uint64_t* __restrict__ bsum) {
  __shared__ uint64_t lds[NWAVE + 1];
  uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_IPT; ++i) {
    uint64_t j = base + (uint64_t)i * NT + threadIdx.x;
    if (j < n) s += (uint64_t)in[j];
  }
  uint64_t tot;
  block_excl_scan(s, lds, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// out[j] = offset(block) + exclusive prefix within block.  Each thread owns
// SCAN_IPT consecutive items.  If `total` is set, the last block writes the
// grand total there.
template <typename T>
__global__ __launch_bounds__(NT) void k_scan_down(const T* __restrict__ in, uint64_t n,
                                                  const uint64_t* __restrict__ boff,
                                                  uint64_t* __restrict__ out,
                                                  uint64_t* __restrict__ total) {
  __shared__ uint64_t lds[NWAVE + 1];
  uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_IPT;
  uint64_t v[SCAN_IPT];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_IPT; ++i) {
    uint64_t j = base + i;
    v[i] = j < n ? (uint64_t)in[j] : 0;
    s += v[i];
  }
  uint64_t tot;
  uint64_t run = block_excl_scan(s, lds, &tot) + (boff ? boff[blockIdx.x] : 0);
#pragma unroll
  for (int i = 0; i < SCAN_IPT; ++i) {
    uint64_t j = base + i;
    if (j < n) out[j] = run;
    run += v[i];
  }
  if (total && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    *total = (boff ? boff[blockIdx.x] : 0) + tot;
}

// Scratch needed by scan_excl_u64 for n items (in u64 words): per level
// nb block sums + nb block offsets + 1, then the level above.
inline uint64_t scan_scratch_words(uint64_t n) {
  uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb <= 1) return 1;
  return 2 * nb + 1 + scan_scratch_words(nb);
}

// Exclusive scan of n items into out (u64).  *d_total (device) receives the sum.
// `scratch` must hold scan_scratch_words(n) u64.
template <typename T>
hipError_t scan_excl_u64(const T* in, uint64_t n, uint64_t* out, uint64_t* d_total,
                         uint64_t* scratch, hipStream_t st) {
  if (n == 0) {
    if (d_total) NLP_HIP(hipMemsetAsync(d_total, 0, 8, st));
    return hipSuccess;
  }
  uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 1) {
    hipLaunchKernelGGL(k_scan_down<T>, dim3(1), dim3(NT), 0, st, in, n, (const uint64_t*)nullptr, out, d_total);
    return hipGetLastError();
  }
  uint64_t* bsum = scratch;
  uint64_t* boff = scratch + nb;
  hipLaunchKernelGGL(k_scan_reduce<T>, dim3((unsigned)nb), dim3(NT), 0, st, in, n, bsum);
  NLP_HIP(hipGetLastError());
  NLP_HIP(scan_excl_u64<uint64_t>(bsum, nb, boff, nullptr, boff + nb + 1, st));
  hipLaunchKernelGGL(k_scan_down<T>, dim3((unsigned)nb), dim3(NT), 0, st, in, n, (const uint64_t*)boff, out, d_total);
  return hipGetLastError();
}

// ---------------------------------------------------------------- load-balanced search
// Given exclusive offsets off[0..items) (non-decreasing, first = 0) and a slot s,
// return the item i with off[i] <= s < off[i+1] (last item if i+1 == items).
__device__ __forceinline__ uint64_t lbs_find(const uint64_t* __restrict__ off, uint64_t items, uint64_t s) {
  uint64_t lo = 0, hi = items;  // upper_bound(s) - 1
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (off[mid] <= s) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

// ---------------------------------------------------------------- stable LSD radix sort
// One pass sorts by an 8-bit digit at bit `shift` of a u64 key.
constexpr int RS_IPT = 4;                  // items per thread per step
constexpr int RS_STEP = NT * RS_IPT;       // 1024 items per step
constexpr int RS_BINS = 256;

__device__ __forceinline__ uint32_t digit_of(uint64_t k, int shift) { return (uint32_t)(k >> shift) & 0xffu; }

// Per-workgroup digit histograms, digit-major: hist[d * nblk + b].
__global__ __launch_bounds__(NT) void k_rs_hist(const uint64_t* __restrict__ keys, uint64_t n, int shift,
                                                uint64_t per_blk, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[RS_BINS];
  h[threadIdx.x] = 0;
  __syncthreads();
  uint64_t b0 = (uint64_t)blockIdx.x * per_blk;
  uint64_t b1 = b0 + per_blk < n ? b0 + per_blk : n;
  for (uint64_t j = b0 + threadIdx.x; j < b1; j += NT) atomicAdd(&h[digit_of(keys[j], shift)], 1u);
  __syncthreads();
  hist[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter.  Items of a workgroup's range are processed in steps of
// RS_STEP, item order = (step, i, thread) with each wave covering 64
// consecutive items per sub-step, so that ranks follow input order exactly.
template <bool HAS_VAL>
__global__ __launch_bounds__(NT) void k_rs_scatter(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                   uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                   uint64_t n, int shift, uint64_t per_blk,
                                                   const uint64_t* __restrict__ hoff) {
  __shared__ uint64_t base[RS_BINS];                  // running global position per digit
  __shared__ uint32_t wcnt[RS_IPT][NWAVE][RS_BINS];   // per (sub-step, wave) digit counts
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  base[t] = hoff[(uint64_t)t * gridDim.x + blockIdx.x];
  uint64_t b0 = (uint64_t)blockIdx.x * per_blk;
  uint64_t b1 = b0 + per_blk < n ? b0 + per_blk : n;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (uint64_t s0 = b0; s0 < b1; s0 += RS_STEP) {
    for (int i = 0; i < RS_IPT; ++i)
      for (int w = 0; w < NWAVE; ++w) wcnt[i][w][t] = 0;
    __syncthreads();
    uint64_t k[RS_IPT];
    uint32_t v[RS_IPT];
    uint32_t d[RS_IPT];
    uint32_t rk[RS_IPT];
    bool ok[RS_IPT];
#pragma unroll
    for (int i = 0; i < RS_IPT; ++i) {
      uint64_t j = s0 + (uint64_t)i * NT + t;  // sub-step i: 256 consecutive items
      ok[i] = j < b1;
      k[i] = ok[i] ? kin[j] : 0;
      if (HAS_VAL) v[i] = ok[i] ? vin[j] : 0;
      d[i] = ok[i] ? digit_of(k[i], shift) : 0;
      // peers: lanes of this wave with the same digit (8 ballots)
      uint64_t peers = __ballot(ok[i]);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        uint64_t bb = __ballot((d[i] >> b) & 1);
        peers &= ((d[i] >> b) & 1) ? bb : ~bb;
      }
      rk[i] = (uint32_t)__popcll(peers & lt);
      if (ok[i] && rk[i] == 0) wcnt[i][wv][d[i]] = (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // thread t owns digit t: exclusive prefix over (sub-step, wave) in order
    {
      uint32_t run = 0;
      for (int i = 0; i < RS_IPT; ++i)
        for (int w = 0; w < NWAVE; ++w) { uint32_t c = wcnt[i][w][t]; wcnt[i][w][t] = run; run += c; }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < RS_IPT; ++i) {
        if (ok[i]) {
          uint64_t pos = base[d[i]] + wcnt[i][wv][d[i]] + rk[i];
          kout[pos] = k[i];
          if (HAS_VAL) vout[pos] = v[i];
        }
      }
      __syncthreads();
      base[t] += run;
    }
    __syncthreads();
  }
}

struct SortScratch {
  uint32_t* hist;     // RS_BINS * max_blocks
  uint64_t* hoff;     // RS_BINS * max_blocks
  uint64_t* scan;     // scan scratch
  uint64_t max_blocks;
};

inline uint64_t rs_blocks(uint64_t n) {
  uint64_t nb = (n + 8 * RS_STEP - 1) / (8 * RS_STEP);  // >= 8 steps per workgroup
  if (nb < 1) nb = 1;
  if (nb > 2048) nb = 2048;
  return nb;
}

// Sort (keys, vals) stably by the bytes listed in `shifts` (least significant
// first).  Ping-pongs between (k0,v0) and (k1,v1); returns in *which the
// buffer index (0/1) holding the result.  vals may be null.
inline hipError_t sort_pairs_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint64_t n,
                                 const int* shifts, int npass, SortScratch& sc, int* which, hipStream_t st) {
  *which = 0;
  if (n <= 1 || npass == 0) return hipSuccess;
  uint64_t nb = rs_blocks(n);
  uint64_t per = (n + nb - 1) / nb;
  per = (per + RS_STEP - 1) / RS_STEP * RS_STEP;
  nb = (n + per - 1) / per;
  uint64_t* ka = k0; uint32_t* va = v0; uint64_t* kb = k1; uint32_t* vb = v1;
  for (int p = 0; p < npass; ++p) {
    hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)nb), dim3(NT), 0, st, ka, n, shifts[p], per, sc.hist);
    NLP_HIP(hipGetLastError());
    NLP_HIP(scan_excl_u64<uint32_t>(sc.hist, (uint64_t)RS_BINS * nb, sc.hoff, nullptr, sc.scan, st));
    if (va)
      hipLaunchKernelGGL(k_rs_scatter<true>, dim3((unsigned)nb), dim3(NT), 0, st, ka, va, kb, vb, n, shifts[p], per, sc.hoff);
    else
      hipLaunchKernelGGL(k_rs_scatter<false>, dim3((unsigned)nb), dim3(NT), 0, st, ka, (const uint32_t*)nullptr, kb,
                         (uint32_t*)nullptr, n, shifts[p], per, sc.hoff);
    NLP_HIP(hipGetLastError());
    uint64_t* tk = ka; ka = kb; kb = tk;
    uint32_t* tv = va; va = vb; vb = tv;
    *which ^= 1;
  }
  return hipSuccess;
}

// ---------------------------------------------------------------- radix select (k-th largest u32)
// State in device memory: sel[0] = prefix (high bits fixed so far), sel[1] = remaining
// rank (1-based among keys matching the prefix), sel[2] = count strictly above
// the final key, sel[3] = the final key, sel[4] = the keys equal to it.
// Digits: 12, 12, 8 bits from the top.
constexpr int SEL_BINS = 4096;

__global__ __launch_bounds__(NT) void k_sel_hist(const uint32_t* __restrict__ keys, const uint64_t* __restrict__ d_n,
                                                 int pass, const uint64_t* __restrict__ sel, uint32_t* __restrict__ ghist) {
  __shared__ uint32_t h[SEL_BINS];
  for (int i = threadIdx.x; i < SEL_BINS; i += NT) h[i] = 0;
  __syncthreads();
  const uint64_t n = *d_n;
  const int hi_bits = pass == 0 ? 0 : (pass == 1 ? 12 : 24);
  const int shift = pass == 0 ? 20 : (pass == 1 ? 8 : 0);
  const uint32_t mask = pass == 2 ? 0xffu : 0xfffu;
  const uint32_t prefix = (uint32_t)sel[0];
  constexpr int UN = 4;  // keys per thread per step, loaded together
  for (uint64_t j0 = (uint64_t)blockIdx.x * NT * UN + threadIdx.x; j0 < n; j0 += (uint64_t)gridDim.x * NT * UN) {
    uint32_t k[UN];
#pragma unroll
    for (int q = 0; q < UN; ++q) k[q] = j0 + (uint64_t)q * NT < n ? keys[j0 + (uint64_t)q * NT] : 0u;
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const bool match = j0 + (uint64_t)q * NT < n && (hi_bits == 0 || (k[q] >> (32 - hi_bits)) == prefix);
      // the lanes sharing lane 0's bin (score keys are skewed: one bin often
      // holds most of a wave) add once; the others one by one
      const uint32_t b = match ? (k[q] >> shift) & mask : 0xffffffffu;
      const uint32_t lead = __builtin_amdgcn_readfirstlane(b);
      const uint64_t same = __ballot(b == lead && lead != 0xffffffffu);
      if (same && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)same) - 1))
        atomicAdd(&h[lead], (uint32_t)__popcll(same));
      if (match && !((same >> (threadIdx.x & 63)) & 1ull)) atomicAdd(&h[b], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SEL_BINS; i += NT)
    if (h[i]) atomicAdd(&ghist[i], h[i]);
}

// Single workgroup: walk the histogram from the top digit down.
__global__ __launch_bounds__(NT) void k_sel_pick(uint32_t* __restrict__ ghist, int pass, uint64_t* __restrict__ sel) {
  __shared__ uint64_t cnt[SEL_BINS];
  __shared__ uint64_t s_part[NT];  // per thread: the sum of its block of bins (blocks from the top bin down)
  const int bins = pass == 2 ? 256 : SEL_BINS;
  const int per = bins / NT;       // 16 or 1
  for (int i = threadIdx.x; i < bins; i += NT) cnt[i] = ghist[i];
  __syncthreads();
  {
    uint64_t sum = 0;
    for (int i = 0; i < per; ++i) sum += cnt[bins - 1 - threadIdx.x * per - i];
    s_part[threadIdx.x] = sum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // walk down from the top bin: whole blocks while their sum stays below the
    // remaining rank, then the block where it is reached bin by bin (bin 0 is
    // never taken off: the walk stops there)
    uint64_t rem = sel[1], above = sel[2];
    int b = 0;
    for (; b < NT - 1; ++b) {
      if (s_part[b] >= rem) break;
      rem -= s_part[b];
      above += s_part[b];
    }
    int d = bins - 1 - b * per;
    for (const int dl = d - per + 1; d > 0 && d >= dl; --d) {
      if (cnt[d] >= rem) break;
      rem -= cnt[d];
      above += cnt[d];
    }
    if (d < 0) d = 0;
    sel[0] = (sel[0] << (pass == 2 ? 8 : 12)) | (uint64_t)d;
    sel[1] = rem;
    sel[2] = above;
    if (pass == 2) {
      sel[3] = sel[0] & 0xffffffffull;
      sel[4] = cnt[d];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SEL_BINS; i += NT) ghist[i] = 0;  // ready for next pass
}

}  // namespace nlp
