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

// grid (ceil((stride - 1) / NT), nb); reads nothing when a header is bad
__global__ __launch_bounds__(NT) void k_merge_blocks(const EdgeOut* __restrict__ blocks, uint64_t stride, uint32_t nb,
                                                     uint64_t k, const unsigned long long* __restrict__ ctr,
                                                     EdgeOut* __restrict__ out) {
  if (ctr[2]) return;
  const uint32_t r = blockIdx.y;
  const EdgeOut* b = blocks + (uint64_t)r * stride;
  const uint64_t n = (uint64_t)b[0].u | ((uint64_t)b[0].v << 32);
  const uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const EdgeOut e = b[1 + i];
  const uint32_t key = score_key(e.score);
  uint64_t pos = i;
  if (pos >= k) return;  // its own block already ranks k entries before it
  for (uint32_t q = 0; q < nb && pos < k; ++q) {
    if (q == r) continue;
    const EdgeOut* o = blocks + (uint64_t)q * stride;
    const uint64_t m = (uint64_t)o[0].u | ((uint64_t)o[0].v << 32);
    pos += q < r ? block_rank<false>(o + 1, m, key) : block_rank<true>(o + 1, m, key);
  }
  if (pos < k) out[pos] = e;
}

}  // namespace nlp
