// multi.hpp -- kernels of the multi-device graph (nlp_graph_create_multi).
//
// The reference runs one OpenMP team over all source vertices
// (predict.hxx:284-339, schedule(dynamic, 2048)) and merges the per-thread
// heaps serially (predict.hxx:431-460).  A multi-device handle instead cuts
// the sources into P contiguous partitions balanced by their wedge work
// (SURVEY §8(e)), predicts each partition's canonical top-k on its device,
// and selects the global top-k histogram-first: key histograms of every
// partition's list give the k-th key and each partition's share, which is a
// prefix of its list; only the shares travel to the first device, where one
// merge kernel (select.hpp k_merge_blocks) orders them.
#pragma once
#include "kernels.hpp"

namespace nlp {

// Partition weight of source u: W(u) (k_hp_work_edges: the wedges of its
// surviving intermediates) times the share (S - u) / S of second hops w > u
// (predict.hxx:221), in 1/1024 steps.
__global__ void k_part_weight(const unsigned long long* __restrict__ wu, uint64_t S, uint64_t* __restrict__ w) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < S; u += (uint64_t)gridDim.x * blockDim.x)
    w[u] = (uint64_t)wu[u] * (((S - u) << 10) / S);
}

// bounds[r - 1] = the first u whose exclusive weight prefix reaches
// r * total / P, r = 1 .. P - 1 (prefix has S + 1 entries, prefix[S] = total).
__global__ void k_split_points(const uint64_t* __restrict__ prefix, uint64_t S, uint32_t P,
                               uint64_t* __restrict__ bounds) {
  const uint32_t r = threadIdx.x + 1;
  if (r >= P) return;
  const uint64_t total = prefix[S];
  const uint64_t target = (total / P) * r + (total % P) * r / P;
  uint64_t lo = 0, hi = S;  // first index with prefix >= target
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (prefix[m] < target) lo = m + 1; else hi = m;
  }
  bounds[r - 1] = lo;
}

// Histogram of the score keys of a canonical (key-descending) edge list from
// its run boundaries -- no atomics, one coalesced read.  Level 0: bins are
// key >> 16; level 1: key & 0xffff of the entries whose key >> 16 == hi.
// first[bin] / last[bin] = 1 + the index of the bin's first / last entry
// (0 = empty); the caller zeroes both.
__global__ void k_sorted_hist(const EdgeOut* __restrict__ e, uint64_t n, int level, uint32_t hi,
                              uint64_t* __restrict__ first, uint64_t* __restrict__ last) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = score_key(e[i].score);
    if (level && (k >> 16) != hi) continue;
    const uint32_t b = level ? (k & 0xffffu) : (k >> 16);
    auto bin_of = [&](uint64_t j, uint32_t* out) -> bool {
      const uint32_t kj = score_key(e[j].score);
      if (level && (kj >> 16) != hi) return false;
      *out = level ? (kj & 0xffffu) : (kj >> 16);
      return true;
    };
    uint32_t nb;
    if (i == 0 || !bin_of(i - 1, &nb) || nb != b) first[b] = i + 1;
    if (i + 1 == n || !bin_of(i + 1, &nb) || nb != b) last[b] = i + 1;
  }
}

}  // namespace nlp
