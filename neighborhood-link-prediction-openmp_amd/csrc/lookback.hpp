// lookback.hpp -- single-pass device-wide primitives with decoupled look-back.
//
// Tiles are claimed with a device-scope atomic ticket (never blockIdx), so a
// tile only ever waits on tiles whose workgroups are already running: the
// look-back cannot deadlock whatever the dispatch order.  Every inter-workgroup
// hand-off is an 8-byte {status, value} word written with ONE agent-scope
// atomic store and read with agent-scope atomic loads -- the data is the flag
// (cdna_hip_programming.md §6 Guideline 16, form R2), so no fences are needed.
// Spins are bounded: a tile that waits too long sets the error word and
// proceeds, and the host reports NLP_ERR_DEVICE instead of hanging the GPU.
//
// State words (tickets, descriptors, histograms) live in one arena that the
// host zeroes with a single hipMemsetAsync at the start of each call.
#pragma once
#include "prims.hpp"
#include <algorithm>

namespace nlp {

constexpr int LB_IPT = 16;             // items per thread
constexpr int LB_TILE = NT * LB_IPT;   // 4096 items per tile (fewer tickets: one word takes ~88 per us)
constexpr uint64_t LB_AGG = 1ull << 62;
constexpr uint64_t LB_PFX = 2ull << 62;
constexpr uint64_t LB_VAL = (1ull << 62) - 1;
constexpr uint32_t LB_SPIN_LIMIT = 1u << 26;

__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Claim a tile id for this workgroup (thread 0 draws, broadcast through LDS).
__device__ __forceinline__ uint32_t lb_ticket(uint32_t* counter, uint32_t* s_tile) {
  if (threadIdx.x == 0) *s_tile = atomicAdd(counter, 1u);
  __syncthreads();
  return *s_tile;
}

// Wave 0 of the workgroup: publish the tile aggregate, look back over the
// predecessors 64 at a time, publish the inclusive prefix; returns the
// exclusive prefix (valid in wave 0 only).
__device__ __forceinline__ uint64_t lb_lookback(uint64_t* desc, uint32_t tile, uint64_t agg, uint32_t* err) {
  const int lane = lane_id();
  if (tile == 0) {
    if (lane == 0) lb_store(&desc[0], LB_PFX | agg);
    return 0;
  }
  if (lane == 0) lb_store(&desc[tile], LB_AGG | agg);
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;  // window [base-63, base]
  uint32_t spins = 0;
  while (true) {
    int64_t j = base - lane;
    uint64_t d = j >= 0 ? lb_load(&desc[j]) : LB_PFX;  // before tile 0: prefix 0
    uint64_t st = d & ~LB_VAL;
    uint64_t pfx = __ballot(st == LB_PFX);
    int first = pfx ? __ffsll((long long)pfx) - 1 : 64;  // nearest prefix in the window
    uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);  // lanes 0..first
    if (__ballot(st == 0) & need) {  // a predecessor nearer than the prefix is not published yet
      if (++spins > LB_SPIN_LIMIT) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t v = (lane <= first && j >= 0) ? (d & LB_VAL) : 0;
    // wave sum
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    excl += v;
    if (pfx) break;
    base -= 64;
  }
  if (lane == 0) lb_store(&desc[tile], LB_PFX | (excl + agg));
  return excl;
}

// Scan state of one single-pass scan: ticket counter + per-tile descriptors.
struct LbState {
  uint32_t* ticket;
  uint64_t* desc;
  uint32_t* err;
};

// Generic single-pass exclusive scan.  F supplies
//   __device__ uint64_t count(uint64_t i) const       value of item i (< n)
//   __device__ void emit(uint64_t i, uint64_t off, uint64_t v) const
// Items are processed LB_IPT consecutive per thread.  The grand total goes to
// *total (written by the last tile).  n is read from device memory.
template <class F>
__global__ __launch_bounds__(NT) void k_lb_scan(F f, const uint64_t* __restrict__ d_n, LbState st,
                                                uint64_t* __restrict__ total) {
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_excl;
  __shared__ uint64_t s_cnt[LB_TILE];  // per-item counts, striped -> blocked -> tile-relative offsets
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + LB_TILE - 1) / LB_TILE;
  if (blockIdx.x >= ntiles) {  // surplus workgroups leave before drawing a ticket
    if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0 && total) *total = 0;
    return;
  }
  const uint32_t tile = lb_ticket(st.ticket, &s_tile);
  const uint64_t base = (uint64_t)tile * LB_TILE;
  // striped (coalesced) evaluation of the counts
#pragma unroll
  for (int i = 0; i < LB_IPT; ++i) {
    uint64_t j = base + (uint64_t)i * NT + threadIdx.x;
    s_cnt[i * NT + threadIdx.x] = j < n ? f.count(j) : 0ull;
  }
  __syncthreads();
  // blocked: thread t owns items [16t, 16t+16) of the tile
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < LB_IPT; ++i) s += s_cnt[threadIdx.x * LB_IPT + i];
  uint64_t agg;
  uint64_t texcl = block_excl_scan(s, s_red, &agg);
  if (wave_id() == 0) {
    uint64_t e = lb_lookback(st.desc, tile, agg, st.err);
    if (threadIdx.x == 0) s_excl = e;
  }
  __syncthreads();
  const uint64_t tbase = s_excl;
  if (tile == ntiles - 1 && threadIdx.x == 0 && total) *total = tbase + agg;
  // rewrite the counts in place with tile-relative exclusive offsets
  uint64_t run = texcl;
  uint64_t cs[LB_IPT];
#pragma unroll
  for (int i = 0; i < LB_IPT; ++i) cs[i] = s_cnt[threadIdx.x * LB_IPT + i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < LB_IPT; ++i) {
    s_cnt[threadIdx.x * LB_IPT + i] = run;
    run += cs[i];
  }
  __syncthreads();
  // striped emission; the count is the difference of consecutive offsets
#pragma unroll
  for (int i = 0; i < LB_IPT; ++i) {
    const int li = i * NT + threadIdx.x;
    uint64_t j = base + li;
    if (j < n) {
      uint64_t o = s_cnt[li];
      uint64_t nx = li + 1 < LB_TILE ? s_cnt[li + 1] : agg;
      f.emit(j, tbase + o, nx - o);
    }
  }
}

inline unsigned lb_grid(uint64_t n_upper) {
  uint64_t g = (n_upper + LB_TILE - 1) / LB_TILE;
  return (unsigned)(g < 1 ? 1 : g);
}

// ---------------------------------------------------------------- onesweep radix sort (u32 keys)
// Stable ascending sort of u32 keys carrying a u32 payload; 4 passes of 8 bits.
// k_os_hist builds all four digit histograms in one read; each k_os_pass
// ranks a tile stably (wave ballot multisplit), publishes per-digit tile counts
// and looks back per digit.
constexpr int OS_IPT = 8;
constexpr int OS_TILE = NT * OS_IPT;  // 2048

__global__ __launch_bounds__(NT) void k_os_hist(const uint32_t* __restrict__ keys, const uint64_t* __restrict__ d_n,
                                                uint32_t* __restrict__ ghist /*4 x 256*/) {
  __shared__ uint32_t h[4][RS_BINS];
  for (int i = threadIdx.x; i < 4 * RS_BINS; i += NT) (&h[0][0])[i] = 0;
  __syncthreads();
  const uint64_t n = *d_n;
  for (uint64_t j = (uint64_t)blockIdx.x * NT + threadIdx.x; j < n; j += (uint64_t)gridDim.x * NT) {
    uint32_t k = keys[j];
    atomicAdd(&h[0][k & 0xff], 1u);
    atomicAdd(&h[1][(k >> 8) & 0xff], 1u);
    atomicAdd(&h[2][(k >> 16) & 0xff], 1u);
    atomicAdd(&h[3][k >> 24], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * RS_BINS; i += NT) {
    uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&ghist[i], c);
  }
}

// desc: ntiles x 256 u64 per pass (zeroed).  Writes keys/vals to the output
// at their stable global positions for this digit.
__global__ __launch_bounds__(NT) void k_os_pass(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                const uint64_t* __restrict__ d_n, int shift,
                                                const uint32_t* __restrict__ ghist /*256 for this pass*/,
                                                uint32_t* __restrict__ ticket, uint64_t* __restrict__ desc,
                                                uint32_t* __restrict__ err) {
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_base[RS_BINS];                // global start of each digit (this tile)
  __shared__ uint32_t s_cnt[OS_IPT][NWAVE][RS_BINS];  // per (sub-step, wave) digit counts -> prefixes
  __shared__ uint64_t s_red[NWAVE + 1];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + OS_TILE - 1) / OS_TILE;
  if (blockIdx.x >= ntiles) return;
  const uint32_t tile = lb_ticket(ticket, &s_tile);
  // digit bases: exclusive scan of the global histogram (thread t = digit t)
  uint64_t tot;
  uint64_t dbase = block_excl_scan(ghist[t], s_red, &tot);
  for (int i = 0; i < OS_IPT; ++i)
    for (int w = 0; w < NWAVE; ++w) s_cnt[i][w][t] = 0;
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t k[OS_IPT], v[OS_IPT], d[OS_IPT], rk[OS_IPT];
  bool ok[OS_IPT];
  const uint64_t b0 = (uint64_t)tile * OS_TILE;
#pragma unroll
  for (int i = 0; i < OS_IPT; ++i) {
    uint64_t j = b0 + (uint64_t)i * NT + t;  // sub-step i covers 256 consecutive items
    ok[i] = j < n;
    k[i] = ok[i] ? kin[j] : 0u;
    v[i] = ok[i] ? vin[j] : 0u;
    d[i] = (k[i] >> shift) & 0xffu;
    uint64_t peers = __ballot(ok[i]);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      uint64_t bb = __ballot((d[i] >> b) & 1);
      peers &= ((d[i] >> b) & 1) ? bb : ~bb;
    }
    rk[i] = (uint32_t)__popcll(peers & lt);
    if (ok[i] && rk[i] == 0) s_cnt[i][wv][d[i]] = (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // thread t owns digit t: exclusive prefix over (sub-step, wave), tile count
  uint32_t run = 0;
  for (int i = 0; i < OS_IPT; ++i)
    for (int w = 0; w < NWAVE; ++w) { uint32_t c = s_cnt[i][w][t]; s_cnt[i][w][t] = run; run += c; }
  // per-digit look-back across tiles
  uint64_t* my = desc + (uint64_t)tile * RS_BINS + t;
  uint64_t excl = 0;
  if (tile == 0) {
    lb_store(my, LB_PFX | run);
  } else {
    lb_store(my, LB_AGG | run);
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    while (j >= 0) {
      uint64_t x = lb_load(desc + (uint64_t)j * RS_BINS + t);
      uint64_t st = x & ~LB_VAL;
      if (st == 0) {
        if (++spins > LB_SPIN_LIMIT) { atomicOr(err, 2u); break; }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      excl += x & LB_VAL;
      if (st == LB_PFX) break;
      --j;
    }
    lb_store(my, LB_PFX | (excl + run));
  }
  s_base[t] = dbase + excl;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < OS_IPT; ++i) {
    if (ok[i]) {
      uint64_t pos = s_base[d[i]] + s_cnt[i][wv][d[i]] + rk[i];
      kout[pos] = k[i];
      vout[pos] = v[i];
    }
  }
}

}  // namespace nlp

namespace nlp {

// ---------------------------------------------------------------- reduce-then-scan
// Three launches, no tickets, no spinning: (A) per-tile aggregates, (S) one
// workgroup scans the aggregates in place, (B) each tile scans itself from its
// prefix and emits.  Used where many tiles are co-resident (a single-pass
// look-back would walk back through aggregates that have no prefix yet).
// F supplies count_a(i) (pass A; may have idempotent side effects), count_b(i)
// (pass B) and emit(i, off, v).  n is read from device memory.
template <class F, int IPT>
__global__ __launch_bounds__(NT) void k_rts_reduce(F f, const uint64_t* __restrict__ d_n, uint64_t* __restrict__ agg) {
  __shared__ uint64_t s_red[NWAVE + 1];
  const uint64_t n = *d_n;
  constexpr int TILE = NT * IPT;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      uint64_t j = t * TILE + (uint64_t)i * NT + threadIdx.x;
      if (j < n) s += f.count_a(j);
    }
    uint64_t tot;
    block_excl_scan(s, s_red, &tot);
    if (threadIdx.x == 0) agg[t] = tot;
  }
}

// One workgroup: exclusive scan of agg[0..ntiles) in place, total -> *total.
template <int IPT>
__global__ __launch_bounds__(1024) void k_rts_aggs(const uint64_t* __restrict__ d_n, uint64_t* __restrict__ agg,
                                                   uint64_t* __restrict__ total) {
  __shared__ uint64_t s_w[16 + 1];
  constexpr int TILE = NT * IPT;
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < ntiles; c0 += 1024) {
    uint64_t j = c0 + threadIdx.x;
    uint64_t x = j < ntiles ? agg[j] : 0;
    uint64_t inc = wave_incl_scan(x);
    if (lane_id() == 63) s_w[threadIdx.x >> 6] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t r = 0;
      for (int w = 0; w < 16; ++w) { uint64_t t = s_w[w]; s_w[w] = r; r += t; }
      s_w[16] = r;
    }
    __syncthreads();
    if (j < ntiles) agg[j] = carry + s_w[threadIdx.x >> 6] + inc - x;
    carry += s_w[16];
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

template <class F, int IPT>
__global__ __launch_bounds__(NT) void k_rts_scan(F f, const uint64_t* __restrict__ d_n, const uint64_t* __restrict__ agg) {
  constexpr int TILE = NT * IPT;
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_cnt[TILE];
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t base = t * TILE;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      uint64_t j = base + (uint64_t)i * NT + threadIdx.x;
      s_cnt[i * NT + threadIdx.x] = j < n ? f.count_b(j) : 0ull;
    }
    __syncthreads();
    uint64_t cs[IPT];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      cs[i] = s_cnt[threadIdx.x * IPT + i];
      s += cs[i];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan(s, s_red, &tot);
    uint64_t run0 = run;
    (void)run0;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      s_cnt[threadIdx.x * IPT + i] = run;
      run += cs[i];
    }
    __syncthreads();
    const uint64_t tb = agg[t];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const int li = i * NT + threadIdx.x;
      uint64_t j = base + li;
      if (j < n) {
        uint64_t o = s_cnt[li];
        uint64_t nx = li + 1 < TILE ? s_cnt[li + 1] : tot;
        f.emit(j, tb + o, nx - o);
      }
    }
    __syncthreads();
  }
}

// Launch the three kernels.  agg must hold ceil(n_upper / (256*IPT)) words.
template <class F, int IPT>
inline hipError_t rts_scan(const F& f, const uint64_t* d_n, uint64_t n_upper, uint64_t* agg, uint64_t* total,
                           hipStream_t st) {
  constexpr int TILE = NT * IPT;
  uint64_t nt = (n_upper + TILE - 1) / TILE;
  unsigned g = (unsigned)std::min<uint64_t>(std::max<uint64_t>(nt, 1), 65535);
  hipLaunchKernelGGL((k_rts_reduce<F, IPT>), dim3(g), dim3(NT), 0, st, f, d_n, agg);
  hipLaunchKernelGGL((k_rts_aggs<IPT>), dim3(1), dim3(1024), 0, st, d_n, agg, total);
  hipLaunchKernelGGL((k_rts_scan<F, IPT>), dim3(g), dim3(NT), 0, st, f, d_n, (const uint64_t*)agg);
  return hipGetLastError();
}

}  // namespace nlp
