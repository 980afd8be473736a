// select.hpp -- device-driven top-k selection and ordering (no host round trip).
//
// The reference keeps per-thread bounded heaps and merges them serially
// (predict.hxx:313-336, 431-460); its choice among equal scores depends on the
// OpenMP schedule.  Here the candidates arrive in
// (u asc, w asc) order; the k-th largest score key is found by a 12/12/8-bit
// radix select, ties at the boundary are kept in arrival order, and a stable
// descending sort by score gives the canonical order
// (score desc, u asc, w asc).  Every kernel reads its sizes from device
// counters, so a prediction is one enqueue with one synchronisation at the end.
#pragma once
#include "group.hpp"

namespace nlp {

// fast-path counter slots (in addition to group.hpp's)
enum { C_SEL_N = 12, C_OUT_N = 13, C_DO_SEL = 14 };

// Arena layout of the fast path, in u64 words.
constexpr uint64_t AR_SEL = 16;         // 8 words of radix-select state
constexpr uint64_t AR_TICKETS = 24;     // 16 u32 tickets
constexpr uint64_t AR_SELHIST = 32;     // 4096 u32
constexpr uint64_t AR_OSHIST = 32 + 2048;  // 1024 u32
constexpr uint64_t AR_DESC = 32 + 2048 + 512;

__global__ void k_sel_init(uint64_t* __restrict__ ctr, uint64_t* __restrict__ sel, uint64_t k) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint64_t n = ctr[C_C];
    const bool d = n > k;
    ctr[C_SEL_N] = d ? n : 0;
    ctr[C_OUT_N] = d ? k : n;
    ctr[C_DO_SEL] = d ? 1 : 0;
    sel[0] = 0;
    sel[1] = k;
    sel[2] = 0;
    sel[3] = 0;
  }
}

__global__ __launch_bounds__(NT) void k_sel_pick2(uint32_t* __restrict__ ghist, int pass, uint64_t* __restrict__ sel,
                                                  const uint64_t* __restrict__ ctr) {
  if (ctr[C_SEL_N] == 0) return;  // nothing to select (histograms stayed zero)
  __shared__ uint64_t cnt[SEL_BINS];
  const int bins = pass == 2 ? 256 : SEL_BINS;
  for (int i = threadIdx.x; i < bins; i += NT) cnt[i] = ghist[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t rem = sel[1], above = sel[2];
    int d = bins - 1;
    for (; d > 0; --d) {
      if (cnt[d] >= rem) break;
      rem -= cnt[d];
      above += cnt[d];
    }
    sel[0] = (sel[0] << (pass == 2 ? 8 : 12)) | (uint64_t)d;
    sel[1] = rem;
    sel[2] = above;
    if (pass == 2) sel[3] = sel[0] & 0xffffffffull;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SEL_BINS; i += NT) ghist[i] = 0;
}

// rank of each tie (key == kth) in arrival order
struct F_Tie {
  const uint32_t* key;
  const uint64_t* sel;
  uint64_t* trank;
  __device__ uint64_t count_a(uint64_t i) const { return key[i] == (uint32_t)sel[3] ? 1 : 0; }
  __device__ uint64_t count_b(uint64_t i) const { return count_a(i); }
  __device__ void emit(uint64_t i, uint64_t off, uint64_t) const { trank[i] = off; }
};

// keep = key > kth, or a tie ranked below the quota; compacted into the T buffers
struct F_Keep {
  const uint32_t* key;
  const uint32_t* u;
  const uint32_t* w;
  const float* s;
  const uint64_t* sel;
  const uint64_t* trank;
  uint32_t* okey;
  uint32_t* ou;
  uint32_t* ow;
  float* os;
  __device__ uint64_t count_a(uint64_t i) const {
    const uint32_t k = key[i], kth = (uint32_t)sel[3];
    return (k > kth || (k == kth && trank[i] < sel[1])) ? 1 : 0;
  }
  __device__ uint64_t count_b(uint64_t i) const { return count_a(i); }
  __device__ void emit(uint64_t i, uint64_t off, uint64_t c) const {
    if (!c) return;
    okey[off] = key[i];
    ou[off] = u[i];
    ow[off] = w[i];
    os[off] = s[i];
  }
};

// One scan for the whole selection: each candidate counts (above << 32 | tie),
// so at candidate i the output slot is above_before + min(ties_before, quota)
// -- ties beyond the quota are dropped, in arrival (u, w) order.
struct F_Sel {
  const uint32_t* key;
  const uint32_t* u;
  const uint32_t* w;
  const float* s;
  const uint64_t* sel;
  uint32_t* okey;
  uint32_t* ou;
  uint32_t* ow;
  float* os;
  __device__ uint64_t count_a(uint64_t i) const {
    const uint32_t k = key[i], kth = (uint32_t)sel[3];
    return k > kth ? (1ull << 32) : (k == kth ? 1ull : 0ull);
  }
  __device__ uint64_t count_b(uint64_t i) const { return count_a(i); }
  __device__ void emit(uint64_t i, uint64_t off, uint64_t c) const {
    if (!c) return;
    const uint64_t above = off >> 32, ties = off & 0xffffffffull, quota = sel[1];
    uint64_t pos;
    if (c >> 32) pos = above + (ties < quota ? ties : quota);
    else if (ties < quota) pos = above + ties;
    else return;
    okey[pos] = key[i];
    ou[pos] = u[i];
    ow[pos] = w[i];
    os[pos] = s[i];
  }
};

struct CandBufs {
  const uint32_t* key;
  const uint32_t* u;
  const uint32_t* w;
  const float* s;
};

// ~key (ascending sort = descending score) and identity payload; the source is
// the selected buffer when a selection ran, else the candidate buffer.
__global__ void k_desc_keys_sel(CandBufs a, CandBufs b, const uint64_t* __restrict__ ctr, uint32_t* __restrict__ k,
                                uint32_t* __restrict__ idx) {
  const uint64_t n = ctr[C_OUT_N];
  const uint32_t* key = ctr[C_DO_SEL] ? b.key : a.key;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    k[i] = ~key[i];
    idx[i] = (uint32_t)i;
  }
}

__global__ void k_gather_sel(const uint32_t* __restrict__ idx, CandBufs a, CandBufs b, const uint64_t* __restrict__ ctr,
                             EdgeOut* __restrict__ out) {
  const uint64_t n = ctr[C_OUT_N];
  const CandBufs c = ctr[C_DO_SEL] ? b : a;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t j = idx[i];
    EdgeOut o;
    o.u = c.u[j];
    o.v = c.w[j];
    o.score = c.s[j];
    out[i] = o;
  }
}

}  // namespace nlp

namespace nlp {

// ---------------------------------------------------------------- block merge (multi-GPU exchange)
// The reference merges its per-thread heaps with a serial k-way heap merge
// (predict.hxx:431-460).  Here the shards' canonical lists arrive as the fixed-
// stride blocks of one all_gather (nlp.h nlp_merge_blocks_device): entry 0 of a
// block is {count lo, count hi, magic}, entries 1..count are sorted by score key
// descending.  Entry i of block r goes to
//   i + sum_{r' < r} #{j in r' : key_j >= key} + sum_{r' > r} #{j in r' : key_j > key},
// which is the canonical order (score desc, then block order = u asc, then the
// block's own (u, w) order).  Consecutive entries of a wave have nearby keys, so
// the lanes' binary searches in another block walk the same cache lines.
constexpr uint32_t BLOCK_MAGIC = 0x4E4C5042u;

__device__ __forceinline__ bool block_count(const EdgeOut* __restrict__ b, uint64_t stride, uint64_t* cnt) {
  const EdgeOut h = b[0];
  const uint64_t c = (uint64_t)h.u | ((uint64_t)h.v << 32);
  *cnt = c;
  return __float_as_uint(h.score) == BLOCK_MAGIC && c < stride;
}

// first j in [0, n) with key(list[j]) < key (STRICT = false) or <= key (STRICT = true)
template <bool STRICT>
__device__ __forceinline__ uint64_t block_rank(const EdgeOut* __restrict__ list, uint64_t n, uint32_t key) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    const uint32_t km = score_key(list[mid].score);
    if (STRICT ? km > key : km >= key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// ctr[0] = sum of counts, ctr[1] = largest count, ctr[2] = 1 when a header is bad
__global__ void k_merge_blocks_check(const EdgeOut* __restrict__ blocks, uint64_t stride, uint32_t nb,
                                     unsigned long long* __restrict__ ctr) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t tot = 0, mx = 0;
    bool bad = false;
    for (uint32_t r = 0; r < nb; ++r) {
      uint64_t c;
      if (!block_count(blocks + (uint64_t)r * stride, stride, &c)) bad = true;
      tot += c;
      mx = c > mx ? c : mx;
    }
    ctr[0] = tot;
    ctr[1] = mx;
    ctr[2] = bad ? 1 : 0;
  }
}

// Dense score keys of the blocks: keys[r * stride + i] = score_key(entry 1 + i of
// block r), so the searches below touch 4-byte keys instead of 12-byte entries.
__global__ __launch_bounds__(NT) void k_merge_keys(const EdgeOut* __restrict__ blocks, uint64_t stride,
                                                   const unsigned long long* __restrict__ ctr,
                                                   uint32_t* __restrict__ keys) {
  if (ctr[2]) return;
  const EdgeOut* b = blocks + (uint64_t)blockIdx.y * stride;
  const uint64_t n = (uint64_t)b[0].u | ((uint64_t)b[0].v << 32);
  const uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
  if (i < n) keys[(uint64_t)blockIdx.y * stride + i] = score_key(b[1 + i].score);
}

// rank of `key` in list[lo, hi): the first j with list[j] < key (lower block,
// LOWER = true: its ties come first) or list[j] <= key (higher block)
template <bool LOWER, typename P>
__device__ __forceinline__ uint64_t merge_rank(P list, uint64_t lo, uint64_t hi, uint32_t key) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    const uint32_t km = list[mid];
    if (LOWER ? km >= key : km > key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// MT_W: windows average ~0.4 MT_T keys on balanced shards (C2 x8: 404, none
// beyond 2048; at 512 a third fall back to global searches, with 2048-entry
// tiles a fifth).
#ifndef MERGE_MT_W
#define MERGE_MT_W 2048
#endif
constexpr int MT_NT = NT, MT_PER = 4, MT_T = MT_NT * MT_PER, MT_G = 8, MT_W = MERGE_MT_W;
static_assert((MT_W & (MT_W - 1)) == 0, "the branchless window search steps by powers of two");

// Bounds of every (block r, tile x, block q), 4 words at bnd[4 * ((r * tiles + x) * nb + q)]:
// {rank of the tile's first (largest) key, rank of its last (smallest) key,
//  window [lo, hi) holding the ranks of the keys strictly between them}.
// The window leaves out the tie runs of the two end keys in q (a count metric
// has long runs of equal scores): for a lower block q those ties rank before
// the first key and after every inner key, for a higher block the other way.
// One thread per search: every dependent chain runs concurrently.
__global__ __launch_bounds__(NT) void k_merge_bounds(const EdgeOut* __restrict__ blocks, uint64_t stride, uint32_t nb,
                                                     uint64_t tiles, const unsigned long long* __restrict__ ctr,
                                                     const uint32_t* __restrict__ keys, uint64_t* __restrict__ bnd) {
  if (ctr[2]) return;
  const uint64_t total = 4 * (uint64_t)nb * tiles * nb;
  for (uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x; g < total; g += (uint64_t)gridDim.x * NT) {
    const uint32_t w = (uint32_t)(g & 3);
    const uint64_t rest = g >> 2;
    const uint32_t q = (uint32_t)(rest % nb);
    const uint64_t rx = rest / nb;
    const uint64_t x = rx % tiles;
    const uint32_t r = (uint32_t)(rx / tiles);
    const EdgeOut hr = blocks[(uint64_t)r * stride];
    const uint64_t n = (uint64_t)hr.u | ((uint64_t)hr.v << 32);
    const uint64_t i0 = x * MT_T;
    uint64_t v = 0;
    if (q != r && i0 < n) {
      const uint64_t i1 = n < i0 + MT_T ? n : i0 + MT_T;
      const uint32_t kf = keys[(uint64_t)r * stride + i0], kl = keys[(uint64_t)r * stride + i1 - 1];
      const EdgeOut h = blocks[(uint64_t)q * stride];
      const uint64_t m = (uint64_t)h.u | ((uint64_t)h.v << 32);
      const uint32_t* kq = keys + (uint64_t)q * stride;
      const bool lower = q < r;
      // w: 0 rank(first), 1 rank(last), 2 window lo, 3 window hi
      if (w == 0) v = lower ? merge_rank<true>(kq, 0, m, kf) : merge_rank<false>(kq, 0, m, kf);
      else if (w == 1) v = lower ? merge_rank<true>(kq, 0, m, kl) : merge_rank<false>(kq, 0, m, kl);
      else if (w == 2) v = merge_rank<true>(kq, 0, m, kf);   // past the ties of the first key
      else v = merge_rank<false>(kq, 0, m, kl);              // before the ties of the last key
      if (w == 3 && kf == kl) v = merge_rank<true>(kq, 0, m, kf);  // one key: empty window
    }
    bnd[g] = v;
  }
}

// grid (ceil((stride - 1) / MT_T), nb), MT_NT threads; reads nothing when a
// header is bad.  A workgroup takes MT_T consecutive entries of block r.  Equal
// keys share their rank in every other block, so ranks are searched once per
// distinct key of the tile (score ties are common: a count metric has few
// distinct scores).  The ranks in block q lie between those of the tile's first
// (largest) and last (smallest) keys: two global searches bound a window of q's
// keys, staged in LDS when it fits MT_W keys, else searched in place.  Blocks
// are taken MT_G at a time.
__global__ __launch_bounds__(MT_NT) void k_merge_blocks(const EdgeOut* __restrict__ blocks, uint64_t stride,
                                                        uint32_t nb, uint64_t k,
                                                        const unsigned long long* __restrict__ ctr,
                                                        const uint32_t* __restrict__ keys,
                                                        const uint64_t* __restrict__ bnd, EdgeOut* __restrict__ out,
                                                        unsigned long long* __restrict__ dbg) {
  __shared__ uint32_t s_win[MT_G][MT_W];
  __shared__ uint32_t s_dkey[MT_T];
  __shared__ uint32_t s_drank[MT_T];  // < 2^32: the host caps the total entries
  __shared__ uint64_t s_b[MT_G][4];
  __shared__ uint64_t s_red[NWAVE + 1];
  if (ctr[2]) return;
  const uint32_t r = blockIdx.y;
  const EdgeOut* b = blocks + (uint64_t)r * stride;
  const uint64_t n = (uint64_t)b[0].u | ((uint64_t)b[0].v << 32);
  const uint64_t i0 = (uint64_t)blockIdx.x * MT_T;
  if (i0 >= n || i0 >= k) return;  // entry i has at least i entries before it
  const uint64_t i1 = n < i0 + MT_T ? n : i0 + MT_T;
  const uint32_t* kr = keys + (uint64_t)r * stride;
  const int t = threadIdx.x;
  // blocked: thread t owns entries i0 + 4t .. +3; distinct keys numbered in order
  uint32_t key[MT_PER];
  EdgeOut ent[MT_PER];
  uint32_t heads = 0;
#pragma unroll
  for (int e = 0; e < MT_PER; ++e) {
    const uint64_t i = i0 + (uint64_t)t * MT_PER + e;
    key[e] = i < i1 ? kr[i] : 0u;
    ent[e] = i < i1 ? b[1 + i] : EdgeOut{0u, 0u, 0.0f};  // issued early: lands while the ranks are searched
    if (i < i1 && (i == i0 || kr[i - 1] != key[e])) ++heads;
  }
  uint64_t nd;
  uint32_t slot = (uint32_t)block_excl_scan(heads, s_red, &nd);
  uint32_t dslot[MT_PER];
#pragma unroll
  for (int e = 0; e < MT_PER; ++e) {
    const uint64_t i = i0 + (uint64_t)t * MT_PER + e;
    if (i < i1 && (i == i0 || kr[i - 1] != key[e])) {
      s_dkey[slot] = key[e];
      s_drank[slot] = 0;
      ++slot;
    }
    dslot[e] = slot - 1;  // the slot of this entry's key
  }
  const uint32_t D = (uint32_t)nd;
  __syncthreads();
  for (uint32_t q0 = 0; q0 < nb; q0 += MT_G) {
    if (t < 4 * MT_G) {  // bounds from k_merge_bounds
      const uint32_t j = t >> 2, q = q0 + j;
      s_b[j][t & 3] = q < nb ? bnd[4 * (((uint64_t)r * gridDim.x + blockIdx.x) * nb + q) + (t & 3)] : 0;
    }
    __syncthreads();
    {
      // stage the windows: the first 2 * MT_NT keys of every window with all loads
      // in flight at once (one round trip), the rare longer tails after
      constexpr int C0 = 2;
      uint32_t wv[MT_G][C0];
#pragma unroll
      for (int j = 0; j < MT_G; ++j) {
        const uint64_t lo = s_b[j][2], len = s_b[j][3] > lo ? s_b[j][3] - lo : 0;
        const uint32_t* kq = keys + (uint64_t)(q0 + j) * stride + lo;
#pragma unroll
        for (int c = 0; c < C0; ++c) {
          const uint32_t x = t + c * MT_NT;
          wv[j][c] = (len <= MT_W && x < len) ? kq[x] : 0u;
        }
      }
#pragma unroll
      for (int j = 0; j < MT_G; ++j) {
        const uint64_t lo = s_b[j][2], len = s_b[j][3] > lo ? s_b[j][3] - lo : 0;
        if (len > MT_W) continue;
#pragma unroll
        for (int c = 0; c < C0; ++c)
          if (t + c * MT_NT < len) s_win[j][t + c * MT_NT] = wv[j][c];
        const uint32_t* kq = keys + (uint64_t)(q0 + j) * stride + lo;
        for (uint32_t x = t + C0 * MT_NT; x < len; x += MT_NT) s_win[j][x] = kq[x];
      }
    }
    __syncthreads();
    // per block: window length, LDS staged or not
    uint32_t wl[MT_G];
    bool inl[MT_G];
#pragma unroll
    for (int j = 0; j < MT_G; ++j) {
      const uint64_t lo = s_b[j][2], len = s_b[j][3] > lo ? s_b[j][3] - lo : 0;
      inl[j] = q0 + j < nb && q0 + j != r && len <= MT_W;
      wl[j] = inl[j] ? (uint32_t)len : 0u;
      if (dbg && t == 0 && q0 + j < nb && q0 + j != r) {  // diagnostics (NLP_DEBUG): windows, fallbacks, distinct keys
        atomicAdd(&dbg[0], 1ull);
        atomicAdd(&dbg[1], (unsigned long long)len);
        if (!inl[j]) atomicAdd(&dbg[2], 1ull);
        if (j == 0) atomicAdd(&dbg[3], (unsigned long long)D);
      }
    }
    for (uint32_t d = t; d < D; d += MT_NT) {
      const uint32_t kd = s_dkey[d];
      const bool inner = d != 0 && d != D - 1;
      // branchless searches of the staged windows, all blocks in lockstep (independent LDS reads per step)
      uint32_t pos[MT_G];
#pragma unroll
      for (int j = 0; j < MT_G; ++j) pos[j] = 0;
#pragma unroll
      for (uint32_t step = MT_W; step >= 1; step >>= 1) {
#pragma unroll
        for (int j = 0; j < MT_G; ++j) {
          if (inner && pos[j] + step <= wl[j]) {
            const uint32_t v = s_win[j][pos[j] + step - 1];
            if (q0 + j < r ? v >= kd : v > kd) pos[j] += step;
          }
        }
      }
      uint64_t add = 0;
#pragma unroll
      for (int j = 0; j < MT_G; ++j) {
        const uint32_t q = q0 + j;
        if (q >= nb || q == r) continue;
        if (d == 0) {
          add += s_b[j][0];
        } else if (d == D - 1) {
          add += s_b[j][1];
        } else if (inl[j]) {
          add += s_b[j][2] + pos[j];
        } else {
          const uint64_t lo = s_b[j][2], hi = s_b[j][3];
          const uint32_t* kq = keys + (uint64_t)q * stride;
          add += q < r ? merge_rank<true>(kq, lo, hi, kd) : merge_rank<false>(kq, lo, hi, kd);
        }
      }
      s_drank[d] += (uint32_t)add;
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < MT_PER; ++e) {
    const uint64_t i = i0 + (uint64_t)t * MT_PER + e;
    const uint64_t pos = i + (i < i1 ? s_drank[dslot[e]] : 0);
    if (i < i1 && pos < k) out[pos] = ent[e];
  }
}

}  // namespace nlp
