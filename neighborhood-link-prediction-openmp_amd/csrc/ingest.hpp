// ingest.hpp -- the reference's input preparation on the device (SURVEY.md
// §8(f) N1 and N2; nlp_ingest_device / nlp_delete_edges_device in nlp.hip).
//
// N1 (main.cxx:241-245): readMtxOmpW keeps every row sorted and unique
// (LazyBitset update, _bitset.hxx:245-262); symmetrizeOmp merges the reverse
// edges of every row with set_union_last_inplace (symmetrize.hxx:72-82,
// _algorithm.hxx:176-214); removeSelfLoopsOmpU drops one (u, u) per row
// (selfLoop.hxx:120-126).  The merge of row v's entries x with its pending
// reverse keys y (sorted, distinct) keeps the last of equal keys only while
// no x entry waits in its deque: walking y in order, keys found in x are
// absorbed until the first key t_v of y that is NOT in x; from there on every
// key of y that is also in x is written twice.  So the row is the
// sorted multiset union in which a key of both x and y appears twice iff it
// is above t_v.  On the device: one sort of all entries tagged (row, key,
// from-y), a per-row minimum of the y keys absent from x (t_v), one keep flag
// per entry, one scan and one scatter -- bit-identical rows, no per-row loop.
//
// N2 (main.cxx:164-169): the deletion draws are sequential by definition
// (one minstd_rand0 engine, batch.hxx:29-58, 99-112) and stay on the host;
// the device resolves each draw's entry, tidies the batch (keep existing,
// sort, unique: batch.hxx:152-208) and applies it (one occurrence per
// deletion: set_difference_inplace, _algorithm.hxx:113-143, batch.hxx:239-247)
// as a flag-scan-scatter compaction of the CSR.
#pragma once
#include "prims.hpp"

namespace nlp {

// (src << 32 | dst) of the file's directed pairs
// Also flags an id above n (*bad = 1): the rows are indexed by id further on
// (k_in_first_absent's t[row], the radix passes cover bits_for(n) bits), so
// one out-of-range id in the file would write past t[] or mis-sort silently.
__global__ void k_in_pairs(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst, uint64_t m,
                           uint64_t n, uint64_t* __restrict__ out, uint32_t* __restrict__ bad) {
  bool oob = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t a = src[i], b = dst[i];
    oob |= a > n || b > n;
    out[i] = ((uint64_t)a << 32) | b;
  }
  if (__ballot(oob) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

// cnt[0] += distinct keys, cnt[1] += distinct keys with high == low half (self loops) of a sorted array
__global__ void k_in_count_distinct(const uint64_t* __restrict__ k, uint64_t n, unsigned long long* __restrict__ cnt) {
  unsigned long long a = 0, b = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (i == 0 || k[i] != k[i - 1]) {
      ++a;
      b += (k[i] >> 32) == (k[i] & 0xffffffffull) ? 1 : 0;
    }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (a) atomicAdd(&cnt[0], a);
    if (b) atomicAdd(&cnt[1], b);
  }
}

// flag[i] = 1 when sorted key i differs from key i - 1 (unique)
__global__ void k_in_first(const uint64_t* __restrict__ k, uint64_t n, uint8_t* __restrict__ flag) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// out[pos[i]] = in[i] where flag[i]
template <typename T>
__global__ void k_in_compact(const T* __restrict__ in, const uint8_t* __restrict__ flag, const uint64_t* __restrict__ pos,
                             uint64_t n, T* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) out[pos[i]] = in[i];
}

// The symmetrize entries of the distinct pairs (u, v): row u gets v from its
// own list x (tag 0) and row v gets u as a pending reverse key y (tag 1):
// (row << 33) | (key << 1) | tag.  Ids < 2^31.
__global__ void k_in_sym_entries(const uint64_t* __restrict__ e, uint64_t ne, uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = e[i] >> 32, v = e[i] & 0xffffffffull;
    out[2 * i] = (u << 33) | (v << 1);
    out[2 * i + 1] = (v << 33) | (u << 1) | 1ull;
  }
}

// the rows of an input that is already symmetric (no symmetrize): tag 0 only
__global__ void k_in_row_entries(const uint64_t* __restrict__ e, uint64_t ne, uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = ((e[i] >> 32) << 33) | ((e[i] & 0xffffffffull) << 1);
}

// t_v = the smallest pending key of row v that is not in x (a tag-1 entry not
// preceded by the same (row, key) with tag 0); t[] starts at 0xffffffff.
__global__ void k_in_first_absent(const uint64_t* __restrict__ k, uint64_t n, uint32_t* __restrict__ t) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = k[i];
    if (!(x & 1ull)) continue;
    if (i > 0 && k[i - 1] == x - 1) continue;  // the key is in x
    atomicMin(&t[x >> 33], (uint32_t)((x >> 1) & 0xffffffffull));
  }
}

// keep flags of the union (the quirk) and of the self-loop removal.  Entries
// are sorted by (row, key, tag): a pending key found in x is kept iff above
// t_row; one copy of (u, u) goes (the tag-0 one, which always exists and
// comes first).  sym = 0: the rows are the tag-0 entries alone.
__global__ void k_in_keep(const uint64_t* __restrict__ k, uint64_t n, const uint32_t* __restrict__ t, int sym,
                          uint8_t* __restrict__ keep) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = k[i];
    const uint64_t row = x >> 33, key = (x >> 1) & 0xffffffffull;
    bool kp;
    if (!(x & 1ull)) kp = row != key;  // removeSelfLoops: the first (u, u) leaves
    else if (!sym) kp = false;
    else if (i > 0 && k[i - 1] == x - 1) kp = key > (uint64_t)t[row];  // in x: written twice above t_row
    else kp = true;
    keep[i] = kp ? 1 : 0;
  }
}

// the kept entries' keys at their positions
__global__ void k_in_scatter_keys(const uint64_t* __restrict__ k, const uint8_t* __restrict__ keep,
                                  const uint64_t* __restrict__ pos, uint64_t n, uint32_t* __restrict__ keys) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (keep[i]) keys[pos[i]] = (uint32_t)((k[i] >> 1) & 0xffffffffull);
}

// off[r] = the output position of row r's first entry = pos[lower_bound(k, r << 33)]
// (pos has n + 1 entries, pos[n] = the total)
__global__ void k_in_offsets(const uint64_t* __restrict__ k, uint64_t n, const uint64_t* __restrict__ pos,
                             uint64_t span, uint64_t* __restrict__ off) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= span; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t target = r << 33;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (k[mid] < target) lo = mid + 1; else hi = mid;
    }
    off[r] = pos[lo];
  }
}

// ---------------------------------------------------------------- N2
// Each drawn (u, index) -> both directions of the entry it names, as (a << 32 | b)
__global__ void k_del_pick(const uint32_t* __restrict__ du, const uint32_t* __restrict__ di, uint64_t nd,
                           const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                           uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nd; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = du[i];
    const uint64_t v = keys[off[u] + di[i]];
    out[2 * i] = (u << 32) | v;
    out[2 * i + 1] = (v << 32) | u;
  }
}

// first occurrence of key v in the sorted row u (or ~0 when absent)
__device__ __forceinline__ uint64_t row_find(const uint64_t* __restrict__ off, const uint32_t* __restrict__ keys,
                                             uint64_t span, uint64_t u, uint32_t v) {
  if (u >= span) return ~0ull;
  uint64_t lo = off[u], hi = off[u + 1];
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (keys[mid] < v) lo = mid + 1; else hi = mid;
  }
  return (lo < off[u + 1] && keys[lo] == v) ? lo : ~0ull;
}

// tidy: keep the sorted deletions that are unique and present in the graph
// (hasEdge, Graph.hxx:185-189); flag[i]
__global__ void k_del_tidy(const uint64_t* __restrict__ d, uint64_t n, const uint64_t* __restrict__ off,
                           const uint32_t* __restrict__ keys, uint64_t span, uint8_t* __restrict__ flag) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = d[i];
    bool f = i == 0 || x != d[i - 1];
    if (f) f = row_find(off, keys, span, x >> 32, (uint32_t)x) != ~0ull;
    flag[i] = f ? 1 : 0;
  }
}

// apply: the first occurrence of each deletion's key in its row leaves
// (removeEdgeIf on a hasVertex target, Graph.hxx:343-346); gone[] starts at 0
__global__ void k_del_mark(const uint64_t* __restrict__ d, uint64_t n, const uint64_t* __restrict__ off,
                           const uint32_t* __restrict__ keys, uint64_t span, uint8_t* __restrict__ gone) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = d[i];
    const uint32_t v = (uint32_t)x;
    if (v == 0 || v >= span) continue;
    const uint64_t p = row_find(off, keys, span, x >> 32, v);
    if (p != ~0ull) gone[p] = 1;
  }
}

__global__ void k_del_keepflag(const uint8_t* __restrict__ gone, uint64_t n, uint8_t* __restrict__ keep) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    keep[i] = gone[i] ? 0 : 1;
}

// off2[u] = pos[off[u]] (pos: exclusive scan of the keep flags, pos[M] = total)
__global__ void k_del_offsets(const uint64_t* __restrict__ off, uint64_t span, const uint64_t* __restrict__ pos,
                              uint64_t* __restrict__ off2) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= span; u += (uint64_t)gridDim.x * blockDim.x)
    off2[u] = pos[off[u]];
}

__global__ void k_del_split(const uint64_t* __restrict__ d, uint64_t n, uint32_t* __restrict__ du,
                            uint32_t* __restrict__ dv) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    du[i] = (uint32_t)(d[i] >> 32);
    dv[i] = (uint32_t)d[i];
  }
}

}  // namespace nlp
