// edgesort.hpp -- the canonical order of a call's links as ONE stable LSD sort
// of 12-byte edge records (gfx950 onesweep passes).
//
// The reference leaves its result in heap-merge order (predict.hxx:431-460)
// and its ties schedule-dependent; the build returns the
// canonical order: score key descending, then u ascending, then w ascending
// (DESIGN.md §2).  That is the ascending order of the composite
//
//     K = (~score_key(s)) << 2vb | u << vb | w          (32 + 2 vb bits)
//
// computed from the record itself, so a record carries no separate key: each
// pass reads (u, w, s), takes its 8-bit digit of K, and writes the record to
// its stable position; the last pass writes the caller's edge array.  The
// round-3 order (two sorts: (u, w) with the key as payload in 7 counted
// passes, then the key in 4, then a gather; C4 JAC H=16: 33.9 ms) moved 8-byte
// keys + payloads through separate histogram and scatter kernels.
//
//   k_es_hist   one read of the records: the 256-bin histogram of every
//               digit (wave-aggregated LDS counts); a digit whose histogram
//               has one bin holding every record is a pass not run
//   k_es_pass   one pass: 5120-record tiles claimed by an ordered ticket; a
//               wave ranks its 640 consecutive records in 10 ballot-multisplit
//               substeps; per digit the tile's count is published, the
//               exclusive prefix over earlier tiles is found by decoupled
//               look-back (u64 descriptors {epoch, status, count}: a pass
//               never clears the previous pass's descriptors, it ignores
//               another epoch); the tile is reordered by digit in LDS and
//               written out in digit runs (consecutive lanes, consecutive
//               12-byte records: coalesced stores; (u, w) staged as one
//               8-byte word, the digit recomputed at the write)
#pragma once
#include "kernels.hpp"
#include "prims.hpp"

namespace nlp {

constexpr int ES_NT = 512;                 // threads per tile
constexpr int ES_IPT = 10;                 // records per thread (tiles of 5120: 71 KB of LDS, two per CU;
                                           // 3072 measured slower, 4096 too)
constexpr int ES_WCH = 64 * ES_IPT;        // 640 consecutive records per wave
constexpr int ES_MAXP = 12;                // digits of a <= 96-bit composite
constexpr uint64_t ES_AGG = 1ull << 46, ES_PFX = 2ull << 46, ES_VAL = ES_AGG - 1;
constexpr uint32_t ES_SPIN_LIMIT = 1u << 26;
constexpr int ES_LBW = 8;                  // predecessors read per look-back round trip

// 8-bit digit `shift` (bit offset) of K; `bits` < 8 for the top digit
__device__ __forceinline__ uint32_t es_digit(uint32_t u, uint32_t w, float s, int vb, int shift) {
  const int lob = 2 * vb;
  const uint32_t hk = ~score_key(s);
  if (shift >= lob) return (hk >> (shift - lob)) & 0xffu;
  const uint64_t lo = ((uint64_t)u << vb) | w;
  uint32_t d = (uint32_t)(lo >> shift);
  if (shift + 8 > lob) d |= hk << (lob - shift);
  return d & 0xffu;
}

// peers of this lane in the wave: the lanes holding the same 8-bit value
__device__ __forceinline__ uint64_t es_peers(uint32_t d, bool ok) {
  uint64_t peers = __ballot(ok);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t bb = __ballot((d >> b) & 1u);
    peers &= ((d >> b) & 1u) ? bb : ~bb;
  }
  return peers;
}

// ghist[p * 256 + d]: records whose digit p (bits 8p..8p+7 of K) is d
__global__ __launch_bounds__(ES_NT) void k_es_hist(const uint32_t* __restrict__ cu, const uint32_t* __restrict__ cw,
                                                   const float* __restrict__ cs, uint64_t n, int vb, int npass,
                                                   uint32_t* __restrict__ ghist) {
  __shared__ uint32_t h[ES_MAXP][256];
  for (int i = threadIdx.x; i < ES_MAXP * 256; i += ES_NT) (&h[0][0])[i] = 0;
  __syncthreads();
  const uint64_t lt = (1ull << lane_id()) - 1ull;
  constexpr int UN = 4;  // records per thread per step, loaded together (the digits wait on one round trip)
  const uint64_t stride = (uint64_t)gridDim.x * ES_NT * UN;
  for (uint64_t j0 = (uint64_t)blockIdx.x * ES_NT * UN; j0 < n; j0 += stride) {  // uniform per wave: ballots below
    uint32_t u[UN], w[UN];
    float s[UN];
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * ES_NT + threadIdx.x;
      const bool ok = j < n;
      u[q] = ok ? cu[j] : 0u;
      w[q] = ok ? cw[j] : 0u;
      s[q] = ok ? cs[j] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const bool ok = j0 + (uint64_t)q * ES_NT + threadIdx.x < n;
      for (int p = 0; p < npass; ++p) {
        const uint32_t d = es_digit(u[q], w[q], s[q], vb, 8 * p);
        const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
        if (__ballot(ok && d != d0) == 0) {  // one digit in the whole wave (the high digits of u often): one atomic
          const uint64_t m = __ballot(ok);
          if (m && lane_id() == 0) atomicAdd(&h[p][d0], (uint32_t)__popcll(m));
        } else if (8 * p + 8 <= 2 * vb) {  // a digit of (u, w): spread over its bins, one LDS atomic per record
          if (ok) atomicAdd(&h[p][d], 1u);
        } else {  // a digit of the score key: few bins, so one atomic per group of equal digits (8 ballots)
          const uint64_t peers = es_peers(d, ok);
          if (ok && (peers & lt) == 0) atomicAdd(&h[p][d], (uint32_t)__popcll(peers));
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < npass * 256; i += ES_NT) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&ghist[i], c);
  }
}

__device__ __forceinline__ void es_publish(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t es_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// FIRST: the input is the candidate columns (cu, cw, cs); else records `in`.
// The output is always records (`out`: the caller's edges on the last pass).
template <bool FIRST, int NTH = ES_NT>  // NTH threads: tiles of NTH x ES_IPT records
__global__ __launch_bounds__(NTH) void k_es_pass(const uint32_t* __restrict__ cu, const uint32_t* __restrict__ cw,
                                                   const float* __restrict__ cs, const EdgeOut* __restrict__ in,
                                                   EdgeOut* __restrict__ out, uint64_t n, int vb, int shift,
                                                   const uint32_t* __restrict__ ghist, uint64_t* __restrict__ desc,
                                                   uint32_t* __restrict__ ticket, uint64_t epoch,
                                                   uint32_t* __restrict__ err) {
  constexpr int ES_NW = NTH / 64, ES_TILE = NTH * ES_IPT;
  static_assert(NTH >= 256, "threads 0-255 own one digit each");
  __shared__ uint64_t s_uw[ES_TILE];       // w << 32 | u: one 8-byte LDS write and read per record
  __shared__ uint32_t s_s[ES_TILE];
  __shared__ uint32_t s_wc[ES_NW][256];   // per wave: running digit counts, then wave prefixes
  __shared__ uint64_t s_gofs[256];        // global position of the tile's first record of each digit
  __shared__ uint32_t s_lofs[256];        // tile position of the first record of each digit
  __shared__ uint32_t s_scan[8];
  __shared__ uint32_t s_tile;
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t ntiles = (n + ES_TILE - 1) / ES_TILE;
  const uint64_t ep = epoch << 48;
  while (true) {
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
    for (int i = t; i < ES_NW * 256; i += NTH) (&s_wc[0][0])[i] = 0;
    __syncthreads();
    const uint64_t tile = s_tile;
    if (tile >= ntiles) break;  // uniform: every wave leaves
    const uint64_t base = tile * ES_TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)ES_TILE, n - base);
    // records of this wave: base + wv * ES_WCH + i * 64 + lane (item order = (wave, substep, lane))
    uint32_t ru[ES_IPT], rw[ES_IPT], rs[ES_IPT], rk[ES_IPT], dg[ES_IPT];
#pragma unroll
    for (int i = 0; i < ES_IPT; ++i) {
      const uint32_t q = (uint32_t)(wv * ES_WCH + i * 64 + lane);
      const bool ok = q < tn;
      const uint64_t j = base + q;
      if (FIRST) {
        ru[i] = ok ? cu[j] : 0u;
        rw[i] = ok ? cw[j] : 0u;
        rs[i] = ok ? __float_as_uint(cs[j]) : 0u;
      } else {
        EdgeOut e{0u, 0u, 0.0f};
        if (ok) e = in[j];
        ru[i] = e.u;
        rw[i] = e.v;
        rs[i] = __float_as_uint(e.score);
      }
    }
#pragma unroll
    for (int i = 0; i < ES_IPT; ++i) {
      const uint32_t q = (uint32_t)(wv * ES_WCH + i * 64 + lane);
      const bool ok = q < tn;
      dg[i] = es_digit(ru[i], rw[i], __uint_as_float(rs[i]), vb, shift);
      const uint64_t peers = es_peers(dg[i], ok);
      const uint64_t below = peers & ((1ull << lane) - 1ull);
      rk[i] = ok ? s_wc[wv][dg[i]] + (uint32_t)__popcll(below) : 0u;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      if (ok && below == 0) s_wc[wv][dg[i]] += (uint32_t)__popcll(peers);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
    __syncthreads();
    // threads 0-255 own digit t: wave prefixes, the tile count, look-back, global base
    uint32_t cnt = 0, gh = 0;
    if (t < 256) {
#pragma unroll
      for (int w = 0; w < ES_NW; ++w) {
        const uint32_t c = s_wc[w][t];
        s_wc[w][t] = cnt;
        cnt += c;
      }
      gh = ghist[t];
      uint64_t* my = desc + tile * 256 + t;
      es_publish(my, ep | (tile == 0 ? ES_PFX : ES_AGG) | (uint64_t)cnt);
    }
    // exclusive scans over the 256 digits (threads 0-255; waves 0-3): tile counts and the pass histogram
    uint32_t lof = 0, gb = 0;
    {
      uint32_t a = cnt, b = gh;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ya = __shfl_up(a, o, 64), yb = __shfl_up(b, o, 64);
        if (lane >= o) { a += ya; b += yb; }
      }
      if (lane == 63 && wv < 4) { s_scan[wv] = a; s_scan[4 + wv] = b; }
      __syncthreads();
      uint32_t pa = 0, pb = 0;
      for (int w = 0; w < wv && w < 4; ++w) { pa += s_scan[w]; pb += s_scan[4 + w]; }
      lof = pa + a - cnt;
      gb = pb + b - gh;
    }
    if (t < 256) {
      uint64_t excl = 0;
      if (tile > 0) {
        // windowed look-back: ES_LBW predecessors per round trip (the tiles in
        // flight have published only their counts, so the nearest inclusive
        // prefix can be hundreds of tiles back), consumed nearest first up to
        // the first inclusive prefix or the first tile not yet counted
        int64_t j = (int64_t)tile - 1;
        uint32_t spins = 0;
        bool fin = false;
        while (!fin) {
          uint64_t x[ES_LBW];
#pragma unroll
          for (int r = 0; r < ES_LBW; ++r)
            x[r] = j - r >= 0 ? es_load(desc + (uint64_t)(j - r) * 256 + t) : (ep | ES_PFX);  // before tile 0: zero
          int used = 0;
          bool blocked = false;
#pragma unroll
          for (int r = 0; r < ES_LBW; ++r) {
            if (fin || blocked) continue;
            const uint64_t st = (x[r] >> 48) == epoch ? (x[r] >> 46) & 3ull : 0ull;
            if (st == 0) {
              blocked = true;
              continue;
            }
            excl += x[r] & ES_VAL;
            ++used;
            fin = st == 2;
          }
          j -= used;
          if (!fin && used == 0) {
            if (++spins > ES_SPIN_LIMIT) { atomicOr(err, 1u); break; }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        es_publish(desc + tile * 256 + t, ep | ES_PFX | (excl + cnt));
      }
      s_gofs[t] = (uint64_t)gb + excl;
      s_lofs[t] = lof;
    }
    __syncthreads();
    // reorder the tile by digit in LDS
#pragma unroll
    for (int i = 0; i < ES_IPT; ++i) {
      const uint32_t q = (uint32_t)(wv * ES_WCH + i * 64 + lane);
      if (q < tn) {
        const uint32_t p = s_lofs[dg[i]] + s_wc[wv][dg[i]] + rk[i];
        s_uw[p] = (uint64_t)rw[i] << 32 | ru[i];
        s_s[p] = rs[i];
      }
    }
    __syncthreads();
    // write the digit runs: consecutive tile positions -> consecutive output records
    for (uint32_t p = (uint32_t)t; p < tn; p += NTH) {
      const uint64_t uw = s_uw[p];
      const uint32_t u = (uint32_t)uw, w = (uint32_t)(uw >> 32), sb = s_s[p];
      const uint32_t d = es_digit(u, w, __uint_as_float(sb), vb, shift);  // recomputed: cheaper than a byte in LDS
      const uint64_t pos = s_gofs[d] + (p - s_lofs[d]);
      out[pos] = EdgeOut{u, w, __uint_as_float(sb)};
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- rank-compressed 8-byte keys
// A call's top k holds few distinct scores (Jaccard / CN at H = 16 on C4: a
// few hundred), so the score key is replaced by its dense rank r among the
// D distinct keys (descending) and the composite
//
//     K8 = r << 2vb | u << vb | w          (bits(D - 1) + 2 vb <= 64 bits)
//
// is sorted instead of K: passes move 8-byte keys instead of 12-byte records,
// and K8 has fewer digits than K (C4: 8 instead of 10 passes).  The last pass
// writes the caller's edges with the score of rank r from a D-entry table.
// The distinct keys are collected in a global open-addressing set of key + 1
// (0 = empty; a key of 0xffffffff is a NaN bit pattern and never occurs),
// filled per workgroup from an LDS set whose lookups are plain reads in the
// steady state (no atomic once a key is in).  Calls with a NaN or zero score
// (several bit patterns behind one key), more than ES_DMAX distinct keys or
// too many bits keep the 12-byte sort.
constexpr uint32_t ES_DCAP = 16384;  // global set slots (<= ES_DMAX keys: load <= 1/4)
constexpr uint32_t ES_DMAX = 4096;   // distinct keys at most (12 rank bits)
constexpr uint32_t ES_LCAP = 4096;   // LDS set slots per workgroup
constexpr int ES_DLOG = 14;
constexpr uint64_t ES8_MIN = 1ull << 16;  // smaller calls keep the 12-byte sort (no extra host round trip)

__device__ __forceinline__ uint32_t es_dhash(uint32_t x, int lg) { return (x * 0x9E3779B1u) >> (32 - lg); }

// gcnt[0]: distinct keys in the global set; gcnt[1]: overflow (the caller keeps the 12-byte sort)
// ckey != nullptr: the keys are read from ckey and only those >= kmin count
// (the final order of the kept candidates straight from the unpruned buffer)
__global__ __launch_bounds__(ES_NT) void k_es_dkeys(const float* __restrict__ cs, uint64_t n, uint32_t* __restrict__ gset,
                                                    uint32_t* __restrict__ gcnt, const uint32_t* __restrict__ ckey,
                                                    uint32_t kmin) {
  __shared__ uint32_t s_set[ES_LCAP];
  __shared__ uint32_t s_n, s_over;
  for (int i = threadIdx.x; i < (int)ES_LCAP; i += ES_NT) s_set[i] = 0;
  if (threadIdx.x == 0) { s_n = 0; s_over = 0; }
  __syncthreads();
  constexpr int LLG = 12;  // log2 ES_LCAP
  constexpr int UN = 8;    // keys per thread loaded together (one round trip, then the LDS probes)
  const uint64_t stride = (uint64_t)gridDim.x * ES_NT * UN;
  for (uint64_t j0 = (uint64_t)blockIdx.x * ES_NT * UN; j0 < n; j0 += stride) {
    uint32_t kq[UN];
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * ES_NT + threadIdx.x;
      kq[q] = j < n ? (ckey ? ckey[j] : score_key(cs[j])) : 0u;
    }
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * ES_NT + threadIdx.x;
      if (j >= n || (ckey && kq[q] < kmin)) continue;
      const uint32_t x = kq[q] + 1u;
      uint32_t h = es_dhash(x, LLG);
      for (uint32_t probe = 0; probe < ES_LCAP; ++probe) {
        const uint32_t cur = s_set[h];  // a plain read: the common case, the key is already in
        if (cur == x) break;
        if (cur == 0) {
          const uint32_t old = atomicCAS(&s_set[h], 0u, x);
          if (old == 0) {
            if (atomicAdd(&s_n, 1u) >= ES_LCAP / 2) s_over = 1;
            break;
          }
          if (old == x) break;
        }
        h = (h + 1) & (ES_LCAP - 1);
      }
    }
    if (s_over) break;  // (racy read is fine: the flag only ever goes up)
  }
  __syncthreads();
  if (s_over) {
    if (threadIdx.x == 0) atomicOr(&gcnt[1], 1u);
    return;
  }
  for (int i = threadIdx.x; i < (int)ES_LCAP; i += ES_NT) {
    const uint32_t x = s_set[i];
    if (!x) continue;
    // once the set has overflowed (more than ES_DMAX keys: the caller keeps the
    // 12-byte sort) nothing more is inserted -- a global set filling up far
    // beyond ES_DMAX made its probe chains long (C4 AA H=32: 66 ms)
    if (__hip_atomic_load(&gcnt[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    uint32_t h = es_dhash(x, ES_DLOG);
    for (uint32_t probe = 0;; ++probe) {
      if (probe >= ES_DCAP) { atomicOr(&gcnt[1], 1u); break; }
      const uint32_t cur = __hip_atomic_load(&gset[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == x) break;
      if (cur == 0) {
        const uint32_t old = atomicCAS(&gset[h], 0u, x);
        if (old == 0) {
          if (atomicAdd(&gcnt[0], 1u) >= ES_DMAX) atomicOr(&gcnt[1], 1u);
          break;
        }
        if (old == x) break;
      }
      h = (h + 1) & (ES_DCAP - 1);
    }
  }
}


// The 8-byte passes split the keys into G ranges of tpw tiles (range g =
// tiles [g tpw, (g + 1) tpw)), one workgroup per range, so that a pass needs no
// look-back: a range's output offsets for digit d are the digit's global
// offset plus the range counts of d in every earlier range, known before the
// pass starts (k_es_off8).  The counts of pass r come from one read of its
// input keys (k_es_cnt8); those of the first pass from k_es_hist8, which reads
// every key anyway.  (Measured on the C4 order: the decoupled look-back of
// k_es_pass took 0.6 of 1.28 ms per pass -- a chain of cross-XCD round trips;
// a pass without it 0.68 ms.)

constexpr int ES8_IPT = 16;  // keys per thread of k_es_pass8
constexpr int ES8_NT = 256;  // its threads: 4096-key tiles (32 KB of keys in LDS, four workgroups per CU)
constexpr int ES8_NTW = 512; // the wide form: 8192-key tiles (64 KB, two workgroups per CU), twice the
                             // keys per digit run and tile -- fewer partial lines at the runs' ends

// Every record's K8 written to `keys` (the passes then read 8-byte keys only:
// the rank lookup is paid once), and the first pass's counts: cnt[d * G + g]
// = the records of range g whose digit at bit shift0 is d, ghist[d] their sum
// over the ranges.  The score -> rank map is rebuilt per workgroup as an LDS hash of
// the D <= ES_DMAX rank scores (rscore[r], rank order): a lookup is an LDS
// probe, not a chain of dependent global loads.  Grid: G.
constexpr int ES8_HLG = 13;  // LDS hash slots: 2 x ES_DMAX
__global__ __launch_bounds__(ES_NT) void k_es_hist8(const uint32_t* __restrict__ cu, const uint32_t* __restrict__ cw,
                                                    const float* __restrict__ cs, uint64_t n, int vb,
                                                    const float* __restrict__ rscore, uint32_t D,
                                                    uint32_t* __restrict__ ghist, uint64_t* __restrict__ keys,
                                                    uint32_t* __restrict__ cnt, uint32_t tpw, uint32_t G,
                                                    int shift0, uint64_t tile) {
  __shared__ uint32_t h[ES_NT / 64][256];
  __shared__ uint32_t s_hk[1 << ES8_HLG];  // score key + 1 (0: empty)
  __shared__ uint16_t s_hr[1 << ES8_HLG];  // its rank
  const int t = threadIdx.x, wv = wave_id();
  for (int i = t; i < ES_NT / 64 * 256; i += ES_NT) (&h[0][0])[i] = 0;
  for (int i = t; i < (1 << ES8_HLG); i += ES_NT) s_hk[i] = 0;
  __syncthreads();
  for (uint32_t r = t; r < D; r += ES_NT) {
    const uint32_t x = score_key(rscore[r]) + 1u;
    uint32_t hh = es_dhash(x, ES8_HLG);
    while (atomicCAS(&s_hk[hh], 0u, x) != 0u) hh = (hh + 1) & ((1u << ES8_HLG) - 1);  // keys distinct, load <= 1/2
    s_hr[hh] = (uint16_t)r;
  }
  __syncthreads();
  auto k8 = [&](uint32_t u, uint32_t w, float sc) {
    const uint32_t x = score_key(sc) + 1u;
    uint32_t hh = es_dhash(x, ES8_HLG);
    while (s_hk[hh] != x) hh = (hh + 1) & ((1u << ES8_HLG) - 1);  // present: every score key has a rank
    return (uint64_t)s_hr[hh] << (2 * vb) | (uint64_t)u << vb | w;
  };
  constexpr int UN = 4;
  const uint64_t lo = min(n, (uint64_t)blockIdx.x * tpw * tile), hi = min(n, lo + (uint64_t)tpw * tile);
  for (uint64_t j0 = lo; j0 < hi; j0 += (uint64_t)ES_NT * UN) {
    uint32_t u[UN], w[UN];
    float s[UN];
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * ES_NT + t;
      const bool ok = j < hi;
      u[q] = ok ? cu[j] : 0u;
      w[q] = ok ? cw[j] : 0u;
      s[q] = ok ? cs[j] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * ES_NT + t;
      if (j < hi) {
        const uint64_t k = k8(u[q], w[q], s[q]);
        keys[j] = k;
        atomicAdd(&h[wv][(uint32_t)(k >> shift0) & 0xffu], 1u);
      }
    }
  }
  __syncthreads();
  if (t < 256) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < ES_NT / 64; ++w) c += h[w][t];
    cnt[(uint64_t)t * G + blockIdx.x] = c;
    if (c) atomicAdd(&ghist[t], c);
  }
}

// The kept candidates (key >= kmin) of an unpruned buffer as K8 keys,
// compacted in any order (the sort orders them): one reservation per
// workgroup and 4096 candidates.  The score -> rank map as in k_es_hist8.
__global__ __launch_bounds__(ES_NT) void k_es_keep8(const uint32_t* __restrict__ ckey, const uint32_t* __restrict__ cu,
                                                    const uint32_t* __restrict__ cw, uint64_t n, uint32_t kmin, int vb,
                                                    const float* __restrict__ rscore, uint32_t D,
                                                    uint64_t* __restrict__ keys, unsigned long long* __restrict__ count) {
  __shared__ uint32_t s_hk[1 << ES8_HLG];
  __shared__ uint16_t s_hr[1 << ES8_HLG];
  __shared__ uint32_t s_wn[ES_NT / 64];
  __shared__ unsigned long long s_base;
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  for (int i = t; i < (1 << ES8_HLG); i += ES_NT) s_hk[i] = 0;
  __syncthreads();
  for (uint32_t r = t; r < D; r += ES_NT) {
    const uint32_t x = score_key(rscore[r]) + 1u;
    uint32_t hh = es_dhash(x, ES8_HLG);
    while (atomicCAS(&s_hk[hh], 0u, x) != 0u) hh = (hh + 1) & ((1u << ES8_HLG) - 1);
    s_hr[hh] = (uint16_t)r;
  }
  __syncthreads();
  constexpr int UN = 8;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (uint64_t j0 = (uint64_t)blockIdx.x * ES_NT * UN; j0 < n; j0 += (uint64_t)gridDim.x * ES_NT * UN) {
    uint32_t x[UN];
    bool kp[UN];
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * ES_NT + t;
      x[q] = j < n ? ckey[j] : 0u;
      kp[q] = j < n && x[q] >= kmin;
      c += (uint32_t)__popcll(__ballot(kp[q]));
    }
    if (lane == 0) s_wn[wv] = c;
    __syncthreads();
    if (t == 0) {
      uint32_t tot = 0;
      for (int w = 0; w < ES_NT / 64; ++w) tot += s_wn[w];
      s_base = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    uint64_t pos = s_base;
    for (int w = 0; w < wv; ++w) pos += s_wn[w];
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const uint64_t m = __ballot(kp[q]);
      if (kp[q]) {
        const uint64_t j = j0 + (uint64_t)q * ES_NT + t;
        uint32_t hh = es_dhash(x[q] + 1u, ES8_HLG);
        while (s_hk[hh] != x[q] + 1u) hh = (hh + 1) & ((1u << ES8_HLG) - 1);  // present: every kept key has a rank
        keys[pos + (uint64_t)__popcll(m & lt)] = (uint64_t)s_hr[hh] << (2 * vb) | (uint64_t)cu[j] << vb | cw[j];
      }
      pos += (uint64_t)__popcll(m);
    }
    __syncthreads();  // s_wn / s_base are rewritten by the next block
  }
}

// cnt[d * G + g]: the keys of range g whose digit (bits shift..) is d, ghist[d]
// their sum over the ranges; ES8_CUN loads in flight per thread
constexpr int ES8_CUN = 8;
__global__ __launch_bounds__(ES_NT) void k_es_cnt8(const uint64_t* __restrict__ keys, uint64_t n, int shift,
                                                   uint32_t* __restrict__ cnt, uint32_t* __restrict__ ghist,
                                                   uint32_t tpw, uint32_t G, uint64_t tile) {
  // four copies per wave (lane & 3), rows padded to 257 words: lanes with the
  // same digit -- the score-rank digits are skewed -- spread over copies and banks
  constexpr int CP = 4, RW = 257;
  __shared__ uint32_t h[ES_NT / 64][CP][RW];
  const int t = threadIdx.x, wv = wave_id(), cp = lane_id() & (CP - 1);
  for (int i = t; i < ES_NT / 64 * CP * RW; i += ES_NT) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const uint64_t lo = min(n, (uint64_t)blockIdx.x * tpw * tile), hi = min(n, lo + (uint64_t)tpw * tile);
  for (uint64_t j0 = lo; j0 < hi; j0 += (uint64_t)ES_NT * ES8_CUN) {
    uint64_t k[ES8_CUN];
#pragma unroll
    for (int q = 0; q < ES8_CUN; ++q) {
      const uint64_t j = j0 + (uint64_t)q * ES_NT + t;
      k[q] = j < hi ? keys[j] : 0ull;
    }
#pragma unroll
    for (int q = 0; q < ES8_CUN; ++q)
      if (j0 + (uint64_t)q * ES_NT + t < hi) atomicAdd(&h[wv][cp][(uint32_t)(k[q] >> shift) & 0xffu], 1u);
  }
  __syncthreads();
  if (t < 256) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < ES_NT / 64; ++w)
#pragma unroll
      for (int z = 0; z < CP; ++z) c += h[w][z][t];
    cnt[(uint64_t)t * G + blockIdx.x] = c;
    if (c) atomicAdd(&ghist[t], c);
  }
}

// off[d * G + g] = (records of digits below d) + (records of digit d in ranges
// below g): grid 256 (one digit each), 1024 threads, G <= 1024
constexpr int ES8_GMAX = 1024;
__global__ __launch_bounds__(ES8_GMAX) void k_es_off8(const uint32_t* __restrict__ cnt,
                                                      const uint32_t* __restrict__ ghist, uint32_t G,
                                                      uint32_t* __restrict__ off) {
  __shared__ uint32_t s_w[ES8_GMAX / 64];
  __shared__ uint32_t s_base;
  const uint32_t d = blockIdx.x, t = threadIdx.x, lane = lane_id(), wv = wave_id();
  if (t < 64) {  // the digit's global offset: ghist[0 .. d)
    uint32_t b = 0;
    for (uint32_t e = t; e < d; e += 64) b += ghist[e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (t == 0) s_base = b;
  }
  const uint32_t c = t < G ? cnt[(uint64_t)d * G + t] : 0u;
  uint32_t a = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(a, o, 64);
    if ((int)lane >= o) a += y;
  }
  if (lane == 63) s_w[wv] = a;
  __syncthreads();
  uint32_t pre = s_base;
  for (uint32_t w = 0; w < wv; ++w) pre += s_w[w];
  if (t < G) off[(uint64_t)d * G + t] = pre + a - c;
}

// One pass over 8-byte keys (k_es_hist8 wrote them), one workgroup per range:
// its tiles in order, each ranked in LDS (in-wave match over the digit's bits,
// per-wave counters, a column scan), gathered in digit order and written to
// the range's running offsets -- the output positions of a stable LSD pass.
// LAST: the output is the caller's edges (the score of rank r from rscore),
// the first nout of them.  No workgroup waits on another.
template <bool LAST, int NTH = ES8_NT>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(4))) void k_es_pass8(
    const float* __restrict__ rscore, const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
    EdgeOut* __restrict__ eout, uint64_t n, int vb, int shift, const uint32_t* __restrict__ off, uint32_t tpw,
    uint32_t G, uint64_t nout) {
  static_assert(NTH >= 256 && NTH % 64 == 0, "threads 0-255 own one digit each");
  constexpr int ES_NW = NTH / 64, ES_TILE = NTH * ES8_IPT, WCH = 64 * ES8_IPT;
  __shared__ uint64_t s_k[ES_TILE];
  __shared__ uint32_t s_wc[ES_NW][256];
  __shared__ uint32_t s_run[256];   // the range's next output position per digit
  __shared__ uint32_t s_lofs[256];  // the tile's first LDS slot per digit
  __shared__ uint32_t s_scan[4];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t ntiles = (n + ES_TILE - 1) / ES_TILE;
  const uint64_t tb = min(ntiles, (uint64_t)blockIdx.x * tpw), te = min(ntiles, tb + tpw);
  const uint64_t vmask = (1ull << vb) - 1ull;
  if (t < 256) s_run[t] = off[(uint64_t)t * G + blockIdx.x];
  uint64_t rk8[ES8_IPT];
  auto load = [&](uint64_t tl) {
    const uint64_t bs = tl * ES_TILE;
    const uint32_t m = tl < te ? (uint32_t)min((uint64_t)ES_TILE, n - bs) : 0u;
#pragma unroll
    for (int i = 0; i < ES8_IPT; ++i) {
      const uint32_t q = (uint32_t)(wv * WCH + i * 64 + lane);
      rk8[i] = q < m ? in[bs + q] : 0ull;
    }
  };
  load(tb);
  for (uint64_t tile = tb; tile < te; ++tile) {
    for (int i = t; i < ES_NW * 256; i += NTH) (&s_wc[0][0])[i] = 0;
    __syncthreads();
    const uint32_t tn = (uint32_t)min((uint64_t)ES_TILE, n - tile * ES_TILE);
    uint32_t rd[ES8_IPT];  // in-wave rank << 8 | digit
#pragma unroll
    for (int i = 0; i < ES8_IPT; ++i) {
      const uint32_t q = (uint32_t)(wv * WCH + i * 64 + lane);
      const bool ok = q < tn;
      const uint32_t dg = (uint32_t)(rk8[i] >> shift) & 0xffu;
      const uint64_t peers = es_peers(dg, ok);
      const uint64_t below = peers & ((1ull << lane) - 1ull);
      rd[i] = (ok ? s_wc[wv][dg] + (uint32_t)__popcll(below) : 0u) << 8 | dg;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      if (ok && below == 0) s_wc[wv][dg] += (uint32_t)__popcll(peers);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
    __syncthreads();
    uint32_t cnt = 0;
    if (t < 256) {
#pragma unroll
      for (int w = 0; w < ES_NW; ++w) {
        const uint32_t c = s_wc[w][t];
        s_wc[w][t] = cnt;
        cnt += c;
      }
    }
    {  // exclusive scan of the tile's digit counts (waves 0-3)
      uint32_t a = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(a, o, 64);
        if (lane >= o) a += y;
      }
      if (lane == 63 && wv < 4) s_scan[wv] = a;
      __syncthreads();
      uint32_t pa = 0;
      for (int w = 0; w < wv && w < 4; ++w) pa += s_scan[w];
      if (t < 256) s_lofs[t] = pa + a - cnt;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ES8_IPT; ++i) {
      const uint32_t q = (uint32_t)(wv * WCH + i * 64 + lane);
      const uint32_t dg = rd[i] & 0xffu;
      if (q < tn) s_k[s_lofs[dg] + s_wc[wv][dg] + (rd[i] >> 8)] = rk8[i];
    }
    __syncthreads();
    load(tile + 1);  // the next tile's keys, in flight through the write-out
#pragma unroll 4
    for (uint32_t p = (uint32_t)t; p < tn; p += NTH) {
      const uint64_t k = s_k[p];
      const uint32_t d = (uint32_t)(k >> shift) & 0xffu;
      const uint64_t pos = (uint64_t)s_run[d] + (p - s_lofs[d]);
      if (LAST) {
        if (pos < nout)  // the first nout in canonical order (the rest: ties beyond the quota)
          eout[pos] = EdgeOut{(uint32_t)((k >> vb) & vmask), (uint32_t)(k & vmask), rscore[k >> (2 * vb)]};
      } else {
        out[pos] = k;
      }
    }
    __syncthreads();
    if (t < 256) s_run[t] += cnt;
  }
}

// ---------------------------------------------------------------- the two-level order
// K8 = rank << 2vb | u << vb | w.  The LSD passes of the two-level order run
// over the (rank, u) bits only -- ceil((rb + vb) / 8) passes instead of
// ceil((rb + 2 vb) / 8): C4 JAC H=16, 5 instead of 8 -- which leaves every run
// of equal (rank, u) contiguous and in the canonical run order, its w in any
// order.  The runs are then put in w order where they lie (w is unique within
// a run: a candidate (u, w) is one link):
//   k_es_runs  tiles of ER_TILE keys plus an rs-key window beyond; a run that
//              starts in the tile and is at most rs long: each key's place is
//              its run's start plus the keys of the run with a smaller w
//              (counted in LDS), the edge written there; a longer run's first
//              key appends the run to the long list
//   k_es_long  a workgroup per long run: its length found by a scan, at most
//              lcap keys sorted in LDS (bitonic over w); a run beyond lcap goes
//              to the very-long list (start, length)
//   very long  (host) the runs gathered as (run index << vb | w), one
//              lsd8_keys sort of them, scattered back (k_es_vgather / k_es_vscatter)
constexpr int ER_IPT = 8;
constexpr uint32_t ER_TILE = (uint32_t)ES_NT * ER_IPT;  // 4096 keys per tile
constexpr uint32_t ER_RSMAX = 64;                        // the window beyond the tile (rs <= ER_RSMAX)
constexpr int EL_NT = 512;
constexpr uint32_t EL_CAPMAX = 8192;                     // keys of a long run sorted in LDS (lcap <= EL_CAPMAX)

__device__ __forceinline__ EdgeOut er_edge(const float* __restrict__ rscore, uint64_t hi, uint32_t w, int vb) {
  return EdgeOut{(uint32_t)(hi & ((1ull << vb) - 1ull)), w, rscore[hi >> vb]};
}

__global__ __launch_bounds__(ES_NT) void k_es_runs(const float* __restrict__ rscore, const uint64_t* __restrict__ keys,
                                                   uint64_t n, int vb, EdgeOut* __restrict__ eout, uint64_t nout,
                                                   uint32_t rs, uint64_t* __restrict__ lst, uint64_t lcap,
                                                   unsigned long long* __restrict__ lcnt) {
  constexpr int NQ = (ER_TILE + ER_RSMAX + 1 + ES_NT - 1) / ES_NT;  // window keys per thread
  __shared__ uint64_t s_k[ER_TILE + ER_RSMAX + 1];
  const uint32_t t = threadIdx.x;
  const uint64_t vmask = (1ull << vb) - 1ull;
  // the window of the tile at a: the key before it, the tile, rs keys beyond
  auto window = [&](uint64_t a, uint64_t* wb, uint32_t* off, uint32_t* wn) {
    *wb = a ? a - 1 : 0;
    *off = a ? 1u : 0u;
    *wn = (uint32_t)min(n - *wb, (uint64_t)(*off + ER_TILE + rs));
  };
  uint64_t pre[NQ];  // the next window's keys, in flight while a tile is worked
  auto load = [&](uint64_t a) {
    if (a >= n) return;
    uint64_t wb;
    uint32_t off, wn;
    window(a, &wb, &off, &wn);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t i = (uint32_t)q * ES_NT + t;
      pre[q] = i < wn ? keys[wb + i] : 0ull;
    }
  };
  load((uint64_t)blockIdx.x * ER_TILE);
  for (uint64_t a = (uint64_t)blockIdx.x * ER_TILE; a < n; a += (uint64_t)gridDim.x * ER_TILE) {
    uint64_t wb;
    uint32_t off, wn;
    window(a, &wb, &off, &wn);
    const bool cut = wb + wn == n;      // the window reaches the last key
    __syncthreads();                    // the previous tile's reads are done
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t i = (uint32_t)q * ES_NT + t;
      if (i < wn) s_k[i] = pre[q];
    }
    __syncthreads();
    load(a + (uint64_t)gridDim.x * ER_TILE);
    const uint32_t tn = (uint32_t)min(n - a, (uint64_t)ER_TILE);
    // every key of a run that starts in the tile, the window's keys beyond it included
#pragma unroll 2
    for (uint32_t x = off + t; x < wn; x += ES_NT) {
      const uint64_t k = s_k[x], hi = k >> vb;
      uint32_t s = x;
      while (s > off && x - s < rs && (s_k[s - 1] >> vb) == hi) --s;
      if (s > 0 && (s_k[s - 1] >> vb) == hi) continue;  // longer than rs behind x, or begun before the tile
      if (s >= off + tn) continue;                      // begun after the tile: the next tile's
      uint32_t e = x + 1;
      while (e < wn && e - s <= rs && (s_k[e] >> vb) == hi) ++e;
      const bool ended = e < wn ? (s_k[e] >> vb) != hi : cut;
      if (ended && e - s <= rs) {
        const uint32_t w = (uint32_t)(k & vmask);
        uint32_t r = 0;
        for (uint32_t j = s; j < e; ++j) r += (uint32_t)(s_k[j] & vmask) < w ? 1u : 0u;
        const uint64_t pos = wb + s + r;
        if (pos < nout) eout[pos] = er_edge(rscore, hi, w, vb);
      } else if (x == s) {
        const unsigned long long i = atomicAdd(lcnt, 1ull);
        if (i < lcap) lst[i] = wb + s;
      }
    }
  }
}

__global__ __launch_bounds__(EL_NT) void k_es_long(const float* __restrict__ rscore, const uint64_t* __restrict__ keys,
                                                   uint64_t n, int vb, EdgeOut* __restrict__ eout, uint64_t nout,
                                                   uint32_t lcap, const uint64_t* __restrict__ lst, uint64_t lmax,
                                                   const unsigned long long* __restrict__ lcnt,
                                                   uint64_t* __restrict__ vlst, uint64_t vcap,
                                                   unsigned long long* __restrict__ vcnt) {
  __shared__ uint32_t s_w[EL_CAPMAX];
  __shared__ uint32_t s_first;
  const uint32_t t = threadIdx.x;
  const uint64_t vmask = (1ull << vb) - 1ull;
  const uint64_t nl = min((uint64_t)*lcnt, lmax);
  for (uint64_t r = blockIdx.x; r < nl; r += gridDim.x) {
    const uint64_t p = lst[r];
    const uint64_t hi = keys[p] >> vb;
    // the run's length by a search of EL_NT probes a round: galloping (the
    // probes lo + (t + 1) step, step x EL_NT while every probe is in the run),
    // then narrowing (step / EL_NT) -- a few rounds whatever the length
    uint64_t lo = 0, step = 1;  // key p + lo is in the run
    uint64_t L = 0;
    while (true) {
      if (t == 0) s_first = EL_NT;
      __syncthreads();
      const uint64_t q = p + lo + (uint64_t)(t + 1) * step;
      if (q >= n || (keys[q] >> vb) != hi) atomicMin(&s_first, t);
      __syncthreads();
      const uint32_t f = s_first;
      __syncthreads();  // every thread read s_first before the next round resets it
      if (f == EL_NT) {  // every probe in the run (only while galloping)
        lo += (uint64_t)EL_NT * step;
        step *= EL_NT;
        continue;
      }
      lo += (uint64_t)f * step;  // in the run; the end within (lo, lo + step]
      if (step == 1) {
        L = lo + 1;
        break;
      }
      step = (step + EL_NT - 1) / EL_NT;  // the probes still reach lo + step
    }
    if (L <= lcap) {
      for (uint32_t j = t; j < L; j += EL_NT) s_w[j] = (uint32_t)(keys[p + j] & vmask);
      const uint32_t n2 = L <= 2 ? 2u : 1u << (32 - __builtin_clz((uint32_t)L - 1u));
      for (uint32_t j = (uint32_t)L + t; j < n2; j += EL_NT) s_w[j] = 0xffffffffu;
      __syncthreads();
      for (uint32_t kk = 2; kk <= n2; kk <<= 1)
        for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
          for (uint32_t i = t; i < n2 / 2; i += EL_NT) {
            const uint32_t lo = ((i & ~(jj - 1)) << 1) | (i & (jj - 1)), hb = lo + jj;
            const uint32_t x = s_w[lo], y = s_w[hb];
            if ((x > y) == ((lo & kk) == 0)) {
              s_w[lo] = y;
              s_w[hb] = x;
            }
          }
          __syncthreads();
        }
      for (uint32_t j = t; j < L; j += EL_NT)
        if (p + j < nout) eout[p + j] = er_edge(rscore, hi, s_w[j], vb);
    } else if (t == 0) {
      const unsigned long long i = atomicAdd(vcnt, 1ull);
      if (i < vcap) {
        vlst[2 * i] = p;
        vlst[2 * i + 1] = L;
      }
    }
    __syncthreads();  // s_w and s_len are rewritten by the next run
  }
}

// the very long runs: vt[3 r] = start, [3 r + 1] length, [3 r + 2] offset in
// the gathered array; a workgroup per run
__global__ void k_es_vgather(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ vt, uint64_t nv, int vb,
                             uint64_t* __restrict__ x) {
  const uint64_t vmask = (1ull << vb) - 1ull;
  for (uint64_t r = blockIdx.x; r < nv; r += gridDim.x) {
    const uint64_t p = vt[3 * r], L = vt[3 * r + 1], o = vt[3 * r + 2];
    for (uint64_t j = threadIdx.x; j < L; j += blockDim.x) x[o + j] = r << vb | (keys[p + j] & vmask);
  }
}

__global__ void k_es_vscatter(const float* __restrict__ rscore, const uint64_t* __restrict__ x,
                              const uint64_t* __restrict__ keys, const uint64_t* __restrict__ vt, uint64_t nv, int vb,
                              EdgeOut* __restrict__ eout, uint64_t nout) {
  const uint64_t vmask = (1ull << vb) - 1ull;
  for (uint64_t r = blockIdx.x; r < nv; r += gridDim.x) {
    const uint64_t p = vt[3 * r], L = vt[3 * r + 1], o = vt[3 * r + 2], hi = keys[p] >> vb;
    for (uint64_t j = threadIdx.x; j < L; j += blockDim.x)
      if (p + j < nout) eout[p + j] = er_edge(rscore, hi, (uint32_t)(x[o + j] & vmask), vb);
  }
}

// n <= 1 or every digit constant: the candidate columns as records, in place order
__global__ void k_es_copy(const uint32_t* __restrict__ cu, const uint32_t* __restrict__ cw,
                          const float* __restrict__ cs, uint64_t n, EdgeOut* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = EdgeOut{cu[i], cw[i], cs[i]};
}

}  // namespace nlp
