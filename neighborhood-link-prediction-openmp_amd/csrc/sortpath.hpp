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
// Inter-workgroup hand-offs: the single-pass scans claim their tiles with an
// ordered ticket (one atomic per tile on a per-launch counter in the arena),
// so every tile a look-back waits on is held by a running workgroup or done,
// whatever the grid size, dispatch order or other work on the device.  Spins
// are bounded and report through the error word like lookback.hpp.  k_sp_runs
// needs no hand-off at all (gapped output, see there).
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
constexpr uint64_t SP_DESC = SP_HORD + HCOPIES * HSTRIDE / 2;    // ticket counters and descriptors follow
// u32 ticket counters of the ticketed launches of one call (zeroed with the arena)
enum { TK_SURV = 0, TK_EXP = 1, TK_RUNS = 2, TK_BUCKET = 3, TK_REC = 8, TK_ORD = 16, SP_NTICK = 24 };

__device__ __forceinline__ uint32_t* hist_copy(uint32_t* h) { return h + (blockIdx.x % HCOPIES) * HSTRIDE; }
__device__ __forceinline__ uint32_t hist_total(const uint32_t* h, uint32_t i) {
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < HCOPIES; ++c) s += h[c * HSTRIDE + i];
  return s;
}

constexpr int EX_IPT = 4;                      // expansion: survivors per thread (blocked)
constexpr int EX_TILE = NT * EX_IPT;           //            survivors per tile
constexpr int RN_IPT = 4;
constexpr int RN_TILE = NT * RN_IPT;           // run scoring (k_sp_scan<F_Runs>): 1024 records per tile
constexpr int RU_IPT = 4;
constexpr int RU_SEG = 64 * RU_IPT;            // k_sp_runs: records per wave = one segment of the gapped layout
constexpr int RU_TILE = NT * RU_IPT;           //            records per workgroup

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

// Call timing without event nodes (an event-record node costs ~4.6 us of GPU
// time inside a replayed graph): ts[0] = ~(earliest workgroup entry of the
// call's first kernel), ts[1] = ~(earliest entry of the hot kernel), ts[2] =
// latest exit of the hot kernel; s_memrealtime ticks (100 MHz).  Minima are
// kept as maxima of the complement so that a zeroed arena is the identity.
enum { TS_FIRST = 0, TS_HOT_IN = 1, TS_HOT_OUT = 2, TS_END = 3, TS_WORDS = 4 };
// host_ctr layout: [0, NCTR) counters, [NCTR, NCTR + TS_WORDS) stamps
constexpr int HC_WORDS = NCTR + TS_WORDS;
// Workgroup 0 only (dispatched first): thousands of same-address atomics
// serialise for microseconds, and a workgroup's later loads wait behind its own.
__device__ __forceinline__ void ts_enter(uint64_t* ts, int slot) {
  if (ts && blockIdx.x == 0 && threadIdx.x == 0)
    atomicMax((unsigned long long*)&ts[slot], (unsigned long long)~__builtin_amdgcn_s_memrealtime());
}
// The end of a kernel = the entry of workgroup 0 of the kernel after it.
__device__ __forceinline__ void ts_mark_end(uint64_t* slot) {
  if (slot && blockIdx.x == 0 && threadIdx.x == 0)
    atomicMax((unsigned long long*)slot, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
// Wedge totals in WSUM_COPIES counters (workgroup b adds into b % WSUM_COPIES)
constexpr int WSUM_COPIES = 16;
__device__ __forceinline__ uint64_t wsum_total(const uint64_t* w) {
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < WSUM_COPIES; ++i) s += w[i];
  return s;
}

// Optional phase stamps for tools/ubench (nullptr in the product): workgroup b
// writes s_memrealtime (100 MHz) of phase i of its first tile to stamp[8 b + i].
__device__ __forceinline__ void sp_stamp(uint64_t* stamp, bool first, int i) {
  if (stamp && first && threadIdx.x == 0) stamp[blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
}
// shader-clock counter beside a stamp (the clock rate = its rate / the 100 MHz stamps')
__device__ __forceinline__ void sp_clock(uint64_t* stamp, int i) {
  if (stamp && threadIdx.x == 0) stamp[blockIdx.x * 8 + i] = __builtin_amdgcn_s_memtime();
}

__device__ __forceinline__ uint64_t lane_mask_lt() {
  const int lane = lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Arena reset of one sort-path call: counters from init, up to three word ranges zeroed.
struct ArenaZero {
  uint64_t lo[3], hi[3];
};
__global__ void k_sp_arena_init(uint64_t* __restrict__ base, ArenaZero z, CtrInit init) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
#pragma unroll
  for (int r = 0; r < 3; ++r)
    for (uint64_t i = z.lo[r] + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < z.hi[r]; i += stride)
      base[i] = i < NCTR ? init.v[i] : 0ull;
}

// ---------------------------------------------------------------- survivors
// Tile = 4 waves x SV_STEPS steps x 256 consecutive vertices (16-byte loads,
// lane l of step i holds vertices base + 256 i + 4 l .. +3); a vertex survives
// when 1 <= deg v <= H (H = 0: IHub, every vertex with edges).  Output
// ascending v.  Tiles come from an ordered ticket (see k_sp_pass).
constexpr int SV_STEPS = 32;
constexpr uint64_t SV_TILE = (uint64_t)NT * 4 * SV_STEPS;  // 32768 vertices per tile

// Ordered tile claim for the persistent scans: thread 0 draws, LDS broadcast.
// s_tk[par] holds the current tile, s_tk[par ^ 1] the prefetched next one
// (draw it after the iteration's first barrier; read after its last).
__device__ __forceinline__ void tk_draw(uint32_t* tick, uint32_t* slot) {
  if (threadIdx.x == 0) *slot = atomicAdd(tick, 1u);
}

__global__ __launch_bounds__(NT) void k_sp_survivors(const uint32_t* __restrict__ deg, uint64_t S, uint32_t H,
                                                     uint32_t* __restrict__ surv, uint64_t* __restrict__ desc,
                                                     uint32_t* __restrict__ tick, uint64_t* __restrict__ ctr,
                                                     uint64_t* __restrict__ stamp, uint64_t* __restrict__ ts) {
  ts_enter(ts, TS_FIRST);
  constexpr int NB = SV_STEPS / 8;  // u32 flag words per lane (8 steps x 4 vertices each)
  __shared__ uint64_t s_w[NWAVE];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_tk[2];
  const int lane = lane_id(), wv = wave_id();
  const uint32_t hm = H ? H : 0xffffffffu;
  const uint64_t ntiles = (S + SV_TILE - 1) / SV_TILE;
  const uint64_t lt = lane_mask_lt();
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  if (blockIdx.x >= ntiles) return;  // only as many claimants as tiles
  tk_draw(tick, &s_tk[0]);
  __syncthreads();
  bool first = true;
  for (int par = 0;; par ^= 1) {
    const uint64_t tile = s_tk[par];
    if (tile >= ntiles) break;
    sp_stamp(stamp, first, 0);
    const uint64_t b0 = tile * SV_TILE + (uint64_t)wv * (256 * SV_STEPS) + 4 * (uint64_t)lane;
    uint32_t bits[NB];
    uint64_t wt = 0;
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      uint4 dv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint64_t v = b0 + (uint64_t)(8 * q + i) * 256;
        if (v + 3 < S) {
          dv[i] = *(const uint4*)(deg + v);
        } else {
          dv[i].x = v < S ? deg[v] : 0u;
          dv[i].y = v + 1 < S ? deg[v + 1] : 0u;
          dv[i].z = v + 2 < S ? deg[v + 2] : 0u;
          dv[i].w = 0u;
        }
      }
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        m |= (uint32_t)(dv[i].x - 1u < hm) << (4 * i);
        m |= (uint32_t)(dv[i].y - 1u < hm) << (4 * i + 1);
        m |= (uint32_t)(dv[i].z - 1u < hm) << (4 * i + 2);
        m |= (uint32_t)(dv[i].w - 1u < hm) << (4 * i + 3);
      }
      bits[q] = m;
      wt += (uint64_t)__popc(m);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wt += __shfl_xor(wt, o, 64);
    if (lane == 0) s_w[wv] = wt;
    __syncthreads();
    tk_draw(tick, &s_tk[par ^ 1]);
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
    for (int i = 0; i < SV_STEPS; ++i) {
      const uint32_t nib = (bits[i / 8] >> (4 * (i % 8))) & 0xfu;
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
    first = false;
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

// cursor[d] starts at the first slot of class d (relative to class 1).  A
// workgroup ranks a tile of DC_IPT x NT vertices per class in LDS and reserves
// each class's run with ONE global atomic (a power-law degree sequence puts
// most vertices in a few low classes: an atomic per vertex serialised on
// those few cursors).  Order inside a class stays arbitrary.
constexpr int DC_IPT = 16;
__global__ __launch_bounds__(NT) void k_deg_class_scatter(const uint32_t* __restrict__ deg, uint64_t S,
                                                          unsigned long long* __restrict__ cursor,
                                                          uint32_t* __restrict__ vbydeg) {
  __shared__ uint32_t cnt[DCAP + 1];
  __shared__ unsigned long long base[DCAP + 1];
  constexpr uint64_t TILE = (uint64_t)NT * DC_IPT;
  for (uint64_t t0 = (uint64_t)blockIdx.x * TILE; t0 < S; t0 += (uint64_t)gridDim.x * TILE) {
    for (uint32_t i = threadIdx.x; i <= DCAP; i += NT) cnt[i] = 0;
    __syncthreads();
    uint32_t d[DC_IPT], r[DC_IPT];
#pragma unroll
    for (int q = 0; q < DC_IPT; ++q) {
      const uint64_t v = t0 + (uint64_t)q * NT + threadIdx.x;
      d[q] = v < S ? deg[v] : 0u;
      if (d[q] >= 1 && d[q] <= DCAP) r[q] = atomicAdd(&cnt[d[q]], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i <= DCAP; i += NT)
      if (cnt[i]) base[i] = atomicAdd(&cursor[i], (unsigned long long)cnt[i]);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < DC_IPT; ++q) {
      const uint64_t v = t0 + (uint64_t)q * NT + threadIdx.x;
      if (d[q] >= 1 && d[q] <= DCAP) vbydeg[base[d[q]] + r[q]] = (uint32_t)v;
    }
    __syncthreads();
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
// Thread t of a tile owns EX_IPT consecutive survivors v (ascending index):
// for each in-edge u -> v with u in [ua, ub), the wedges (u, v, w) with w in
// N(v), w > u.  Records land in survivor order (single-pass scan over
// ticketed tiles).  A survivor whose N(v) and I(v) both fit EX_REG entries is
// enumerated from registers (no search: one round of independent loads);
// larger ones walk I(v) with an upper_bound into N(v).  Records beyond capW
// are not written; the total still goes to ctr[C_W] (the host regrows and
// reruns).  HIST: also the histogram of record-key digit (key >> hshift) & 255
// (the MSD pass), accumulated per workgroup in LDS; the last tile stores the
// sortable record count ctr[C_WSORT] (0 and F_OVERFLOW when the records exceed
// capW).
constexpr int EX_REG = 8;

struct ExSurv {
  uint32_t v, d, nin;
  uint64_t a;             // toff[v]
  const uint32_t* nv;     // N(v)
  bool reg;
  uint32_t N[EX_REG], I[EX_REG];
};

__device__ __forceinline__ void ex_load(const GraphView& g, uint32_t v, ExSurv& x) {
  x.v = v;
  x.d = g.deg[v];
  x.a = g.toff[v];
  x.nin = (uint32_t)(g.toff[v + 1] - x.a);
  x.nv = g.keys + g.off[v];
  x.reg = x.d <= EX_REG && x.nin <= EX_REG;
  if (x.reg) {
#pragma unroll
    for (int q = 0; q < EX_REG; ++q) {
      x.N[q] = q < (int)x.d ? x.nv[q] : 0u;
      x.I[q] = q < (int)x.nin ? g.tkeys[x.a + q] : 0u;
    }
  }
}

// Every wedge (u, v = x.v, w) of survivor x with u in [ua, ub) and w > u, in
// the order (u ascending over I(v), w ascending over N(v)): put(u, w).
template <class Put>
__device__ __forceinline__ void ex_enum(const GraphView& g, const ExSurv& x, uint64_t ua, uint64_t ub, Put&& put) {
  if (x.reg) {
#pragma unroll
    for (int p = 0; p < EX_REG; ++p) {
      const uint32_t u = x.I[p];
      if (p < (int)x.nin && u >= ua && u < ub) {
#pragma unroll
        for (int q = 0; q < EX_REG; ++q)
          if (q < (int)x.d && x.N[q] > u) put(u, x.N[q]);
      }
    }
  } else {
    for (uint32_t p = 0; p < x.nin; ++p) {
      const uint32_t u = g.tkeys[x.a + p];
      if (u < ua || u >= ub) continue;
      for (uint32_t k = upper_bound_u32(x.nv, x.d, u); k < x.d; ++k) put(u, x.nv[k]);
    }
  }
}

// Number of wedges of survivor x (same set as ex_enum).
__device__ __forceinline__ uint64_t ex_count(const GraphView& g, const ExSurv& x, uint64_t ua, uint64_t ub) {
  uint64_t c = 0;
  if (x.reg) {
#pragma unroll
    for (int p = 0; p < EX_REG; ++p) {
      const uint32_t u = x.I[p];
      if (p < (int)x.nin && u >= ua && u < ub) {
#pragma unroll
        for (int q = 0; q < EX_REG; ++q) c += (q < (int)x.d && x.N[q] > u) ? 1u : 0u;
      }
    }
  } else {
    for (uint32_t p = 0; p < x.nin; ++p) {
      const uint32_t u = g.tkeys[x.a + p];
      if (u >= ua && u < ub) c += x.d - upper_bound_u32(x.nv, x.d, u);
    }
  }
  return c;
}

// The degree-class index's (deg v << 48 | off v) words (k_sv_pack, built once
// per graph) give a survivor's row in the same round trip as its id.
// Symmetric graphs: I(v) = N(v).  Asymmetric graphs (the reference's ingest
// keeps duplicate entries, and a deletion removes one occurrence per row): a
// second word (|I(v)| << 48 | toff v) per entry, unless some in-degree reaches
// 2^16 (flag[0] set; the host then drops both packs).
constexpr int SV_PACK_SHIFT = 48;
__global__ void k_sv_pack(const uint32_t* __restrict__ vbydeg, uint64_t n, const uint64_t* __restrict__ off,
                          const uint32_t* __restrict__ deg, uint64_t* __restrict__ pack,
                          const uint64_t* __restrict__ toff = nullptr, uint64_t* __restrict__ pack_in = nullptr,
                          uint32_t* __restrict__ flag = nullptr) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = vbydeg[i];
    pack[i] = ((uint64_t)deg[v] << SV_PACK_SHIFT) | off[v];
    if (pack_in) {
      const uint64_t a = toff[v], nin = toff[v + 1] - a;
      if (nin >= (1ull << (64 - SV_PACK_SHIFT))) flag[0] = 1u;
      pack_in[i] = (nin << SV_PACK_SHIFT) | a;
    }
  }
}

__device__ __forceinline__ void ex_load_packed(const GraphView& g, uint32_t v, uint64_t pk, ExSurv& x,
                                               const uint64_t* pk_in = nullptr) {
  x.v = v;
  x.d = (uint32_t)(pk >> SV_PACK_SHIFT);
  x.nv = g.keys + (pk & ((1ull << SV_PACK_SHIFT) - 1));
  if (pk_in) {
    x.nin = (uint32_t)(*pk_in >> SV_PACK_SHIFT);
    x.a = *pk_in & ((1ull << SV_PACK_SHIFT) - 1);
  } else {
    x.nin = x.d;
    x.a = pk & ((1ull << SV_PACK_SHIFT) - 1);
  }
  x.reg = x.d <= EX_REG && x.nin <= EX_REG;
  if (x.reg) {
#pragma unroll
    for (int q = 0; q < EX_REG; ++q) {
      x.N[q] = q < (int)x.d ? x.nv[q] : 0u;
      x.I[q] = pk_in ? (q < (int)x.nin ? g.tkeys[x.a + q] : 0u) : x.N[q];
    }
  }
}

__device__ __forceinline__ uint64_t ex_key(uint32_t u, uint32_t w, uint64_t ua, int wbits) {
  return ((uint64_t)(u - ua) << wbits) | w;
}

__device__ __forceinline__ void ex_empty(const GraphView& g, ExSurv& x) {
  x.nin = 0;
  x.d = 0;
  x.reg = true;
  x.v = 0;
  x.a = 0;
  x.nv = g.keys;
}

// wedges of survivor x written from `pos` (HIST: MSD digit histogram in LDS)
template <bool HIST>
__device__ __forceinline__ void ex_write(const GraphView& g, const ExSurv& x, uint64_t ua, uint64_t ub, int wbits,
                                         uint64_t pos, uint64_t* __restrict__ rkey, uint32_t* __restrict__ rval,
                                         uint32_t* s_h, int hshift, int hdigits) {
  ex_enum(g, x, ua, ub, [&](uint32_t u, uint32_t w) {
    const uint64_t key = ex_key(u, w, ua, wbits);
    rkey[pos] = key;
    rval[pos] = x.v;
    if (HIST) {
      atomicAdd(&s_h[(uint32_t)(key >> hshift) & 0xffu], 1u);
      if (hdigits > 1) atomicAdd(&s_h[RS_BINS + ((uint32_t)(key >> (hshift + 8)) & 0xffu)], 1u);
    }
    ++pos;
  });
}

template <bool HIST, int IPT = EX_IPT>
__global__ __launch_bounds__(NT) void k_sp_expand(GraphView g, uint64_t ua, uint64_t ub, int wbits,
                                                  const uint32_t* __restrict__ surv, uint64_t capW,
                                                  uint64_t* __restrict__ rkey, uint32_t* __restrict__ rval,
                                                  uint64_t* __restrict__ desc, uint32_t* __restrict__ tick,
                                                  uint64_t* __restrict__ ctr, int hshift, uint32_t* __restrict__ ghist,
                                                  int hdigits, uint64_t* __restrict__ ts) {
  ts_enter(ts, TS_FIRST);
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_h[HIST ? 2 * RS_BINS : 1];
  __shared__ uint32_t s_tk[2];
  constexpr uint64_t TILE = (uint64_t)NT * IPT;
  const uint64_t n = ctr[C_NV];
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  uint32_t* err = (uint32_t*)&ctr[C_FLAGS] + 1;
  if (blockIdx.x >= ntiles) return;  // only as many claimants as tiles
  if (HIST) {
    s_h[threadIdx.x] = 0;
    s_h[RS_BINS + threadIdx.x] = 0;
  }
  tk_draw(tick, &s_tk[0]);
  __syncthreads();
  for (int par = 0;; par ^= 1) {
    const uint64_t tile = s_tk[par];
    if (tile >= ntiles) break;
    const uint64_t i0 = tile * TILE + (uint64_t)threadIdx.x * IPT;
    ExSurv x[IPT];
    uint64_t c[IPT], sum = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      if (i0 + j < n) ex_load(g, surv[i0 + j], x[j]);
      else ex_empty(g, x[j]);
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      c[j] = ex_count(g, x[j], ua, ub);
      sum += c[j];
    }
    uint64_t agg;
    uint64_t pos = block_excl_scan(sum, s_red, &agg);  // syncs
    tk_draw(tick, &s_tk[par ^ 1]);
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
    pos += s_excl;
    if (sum && pos + sum <= capW) {
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        if (c[j]) ex_write<HIST>(g, x[j], ua, ub, wbits, pos, rkey, rval, s_h, hshift, hdigits);
        pos += c[j];
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

// ---------------------------------------------------------------- direct bucket emission
// The count metrics do not depend on the order of the wedges inside a (u, w)
// run, so their records can go straight to their bucket (the key's top
// `dbits` bits, key >> hshift) in any order: k_sp_excount counts the records
// per bucket (DX_COPIES histogram copies) and in total (ctr[C_W]);
// k_sp_exemit reserves one slot range per (workgroup, bucket) with a global
// cursor and writes the records there.  No look-back and no MSD pass;
// k_sp_group then sorts balanced ranges of whole buckets by key.  One
// survivor per thread, no hand-off between workgroups.
constexpr int DX_MAXBITS = 12;
constexpr uint32_t DX_MAXB = 1u << DX_MAXBITS;  // buckets at most
constexpr int DX_COPIES = 4;                     // histogram copies (contention of the adds)

__global__ __launch_bounds__(NT) void k_sp_excount(GraphView g, uint64_t ua, uint64_t ub, int wbits,
                                                   const uint32_t* __restrict__ surv, uint64_t* __restrict__ ctr,
                                                   int hshift, int dbits, uint32_t* __restrict__ ghist,
                                                   uint64_t* __restrict__ wsum, uint64_t* __restrict__ ts) {
  ts_enter(ts, TS_FIRST);
  __shared__ uint32_t s_h[DX_MAXB];
  __shared__ uint64_t s_red[NWAVE];
  const int t = threadIdx.x;
  const uint32_t nb = 1u << dbits, bm = nb - 1;
  const uint64_t n = ctr[C_NV];
  if ((uint64_t)blockIdx.x * NT >= n) return;
  for (uint32_t i = t; i < nb; i += NT) s_h[i] = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * NT + t;
  ExSurv x;
  if (i < n) ex_load(g, surv[i], x);
  else ex_empty(g, x);
  uint64_t c = 0;
  ex_enum(g, x, ua, ub, [&](uint32_t u, uint32_t w) {
    atomicAdd(&s_h[(uint32_t)(ex_key(u, w, ua, wbits) >> hshift) & bm], 1u);
    ++c;
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane_id() == 0) s_red[wave_id()] = c;
  __syncthreads();
  uint32_t* hc = ghist + (blockIdx.x % DX_COPIES) * DX_MAXB;
  for (uint32_t b = t; b < nb; b += NT) {
    const uint32_t h = s_h[b];
    if (h) atomicAdd(&hc[b], h);
  }
  if (t == 0) {
    uint64_t tot = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) tot += s_red[w];
    if (tot) atomicAdd((unsigned long long*)&wsum[blockIdx.x % WSUM_COPIES], (unsigned long long)tot);
  }
}

__global__ __launch_bounds__(NT) void k_sp_exemit(GraphView g, uint64_t ua, uint64_t ub, int wbits,
                                                  const uint32_t* __restrict__ surv, uint64_t capW,
                                                  uint64_t* __restrict__ rkey, uint32_t* __restrict__ rval,
                                                  uint64_t* __restrict__ ctr, int hshift, int dbits,
                                                  const uint32_t* __restrict__ ghist, uint32_t* __restrict__ bcur,
                                                  const uint64_t* __restrict__ wsum) {
  constexpr uint32_t PER = DX_MAXB / NT;  // buckets per thread in the start scan
  __shared__ uint32_t s_h[DX_MAXB];       // records per bucket, then the next free slot per bucket
  __shared__ uint32_t s_start[DX_MAXB];
  __shared__ uint64_t s_red[NWAVE + 1];
  const int t = threadIdx.x;
  const uint32_t nb = 1u << dbits, bm = nb - 1;
  const uint64_t n = ctr[C_NV];
  if ((uint64_t)blockIdx.x * NT >= n) return;
  const uint64_t W = wsum_total(wsum);
  const bool fits = W <= capW;
  if (blockIdx.x == 0 && t == 0) {
    ctr[C_W] = W;
    ctr[C_WSORT] = fits ? W : 0;
    if (!fits) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_OVERFLOW);
  }
  if (!fits) return;
  // bucket starts: exclusive scan of the summed histogram copies (thread t: PER consecutive buckets)
  {
    const uint32_t per = (nb + NT - 1) / NT;
    uint32_t hv[PER], sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const uint32_t b = t * per + q;
      uint32_t h = 0;
      if (q < per && b < nb) {
#pragma unroll
        for (int cpy = 0; cpy < DX_COPIES; ++cpy) h += ghist[cpy * DX_MAXB + b];
      }
      hv[q] = h;
      sum += h;
    }
    uint64_t tot;
    uint32_t run = (uint32_t)block_excl_scan(sum, s_red, &tot);  // syncs
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const uint32_t b = t * per + q;
      if (q < per && b < nb) {
        s_start[b] = run;
        s_h[b] = 0;
      }
      run += hv[q];
    }
  }
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * NT + t;
  ExSurv x;
  if (i < n) ex_load(g, surv[i], x);
  else ex_empty(g, x);
  ex_enum(g, x, ua, ub, [&](uint32_t u, uint32_t w) {
    atomicAdd(&s_h[(uint32_t)(ex_key(u, w, ua, wbits) >> hshift) & bm], 1u);
  });
  __syncthreads();
  for (uint32_t b = t; b < nb; b += NT) {
    const uint32_t c = s_h[b];
    s_h[b] = s_start[b] + (c ? atomicAdd(&bcur[b], c) : 0u);
  }
  __syncthreads();
  ex_enum(g, x, ua, ub, [&](uint32_t u, uint32_t w) {
    const uint64_t key = ex_key(u, w, ua, wbits);
    const uint32_t pos = atomicAdd(&s_h[(uint32_t)(key >> hshift) & bm], 1u);
    rkey[pos] = key;
    rval[pos] = x.v;
  });
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

// ---------------------------------------------------------------- onesweep pass
constexpr int OS_NT = 1024;                      // threads per tile: 16 waves
constexpr int OS_NT_C = OS_NT;
constexpr int OS_NW = OS_NT / 64;
constexpr int OS2_IPT = 4;                       // keys per thread
constexpr int OS2_TILE = OS_NT * OS2_IPT;        // 4096 keys per tile
constexpr int OS_LBW = 64;                       // predecessors read per look-back round trip
constexpr uint32_t OS_AGG = 1u << 30, OS_PFX = 2u << 30, OS_VAL = OS_AGG - 1;
constexpr uint64_t SP_MAX_N = (1ull << 30) - 1;  // u32 descriptors: 30-bit counts

__device__ __forceinline__ void st_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefixes of ND digits d[k] over tiles [0, tile): per digit, the
// sum of the nearest predecessors' values back to (and including) the first
// inclusive prefix.  W predecessors per digit per round trip, all loads of a
// round issued before any is inspected; only existing predecessors are read
// (32-bit offsets from the descriptor base, nb descriptors per tile), the
// window beyond tile 0 reads as a zero prefix.
template <int ND, int W>
__device__ __forceinline__ void os_lookback(const uint32_t* desc, uint32_t nb, uint64_t tile, const uint32_t (&d)[ND],
                                            uint32_t (&excl)[ND], uint32_t* err) {
  int32_t j[ND];  // tiles < 2^22: SP_MAX_N / OS2_TILE
  bool done[ND];
#pragma unroll
  for (int q = 0; q < ND; ++q) {
    excl[q] = 0;
    j[q] = (int32_t)tile - 1;
    done[q] = j[q] < 0;
  }
  uint32_t spins = 0;
  while (true) {
    bool all = true;
#pragma unroll
    for (int q = 0; q < ND; ++q) all &= done[q];
    if (all) break;
    uint32_t x[ND][W];
#pragma unroll
    for (int q = 0; q < ND; ++q)
#pragma unroll
      for (int r = 0; r < W; ++r)
        x[q][r] = (!done[q] && r <= j[q]) ? ld_u32(&desc[(uint32_t)(j[q] - r) * nb + d[q]]) : OS_PFX;
    bool moved = false;
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      if (done[q]) continue;
      int used = 0;
      bool fin = false, blocked = false;
#pragma unroll
      for (int r = 0; r < W; ++r) {
        if (!fin && !blocked) {
          const uint32_t st = x[q][r] >> 30;
          if (st == 0) {
            blocked = true;
          } else {
            excl[q] += x[q][r] & OS_VAL;
            ++used;
            fin = st == 2;
          }
        }
      }
      done[q] = fin;
      j[q] -= used;
      moved |= used > 0;
    }
    if (!moved) {
      if (++spins > LB_SPIN_LIMIT) {
        atomicOr(err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

// Digit geometry of a counting pass with DB-bit digits: NB bins; the digit
// histograms of the later passes in HC copies of HS words (digit p of a copy
// at p NB); per-wave counts fit u16 at 11 bits (<= 64 IPT per wave).
template <int DB>
struct PassDigits {
  static constexpr int NB = 1 << DB;
  static constexpr int HC = DB == 8 ? HCOPIES : 4;
  static constexpr uint32_t HS = DB == 8 ? HSTRIDE : 3u * (1u << DB);
  static constexpr int ND = NB > OS_NT_C ? NB / OS_NT_C : 1;  // digits per owner thread
  static constexpr int LBW = ND == 1 ? 64 : 32;                // look-back window per digit
  static constexpr int NHD = (32 - DB + DB - 1) / DB;          // later digits of a 32-bit key
  using CT = typename std::conditional<(DB > 8), uint16_t, uint32_t>::type;
};
template <int DB>
__device__ __forceinline__ uint32_t* hist_copy_db(uint32_t* h) {
  return h + (blockIdx.x % PassDigits<DB>::HC) * PassDigits<DB>::HS;
}
template <int DB>
__device__ __forceinline__ uint32_t hist_total_db(const uint32_t* h, uint32_t i) {
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < PassDigits<DB>::HC; ++c) s += h[c * PassDigits<DB>::HS + i];
  return s;
}

// One stable counting pass on digit (key >> shift) & 255 (onesweep, after
// Adinets & Merrill, restated for gfx950): 1024-thread tiles, wave w owning
// 64 * IPT consecutive keys, so a wave ranks its keys in IPT ballot-multisplit
// substeps (short dependent chain); threads 0-255 then own one digit each for
// the wave prefix, the look-back and the inclusive prefix.  Tiles are claimed
// with an ordered ticket (one atomic per tile on a per-launch counter): a tile
// only waits on tiles held by running workgroups -- no co-residency
// assumption, any grid size.  Descriptors are u32 {status:2, count:30} at
// desc[tile * 256 + digit], each written by one agent-scope atomic store and
// read by agent-scope atomic loads (the data is the flag: no fences).
//
// GAPPED (GAP_SEGMENTS): the input is k_sp_runs' layout -- slot j is valid
// when j < n and j % RU_SEG < seg_cnt[j / RU_SEG] -- and the pass writes the
// number of valid keys (the candidate count) to *tot_out.
// NEXT_HIST: also count digits 1..3 (shift 8, 16, 24) of the input keys into
// the histogram copies at nhist (the first pass of a 32-bit sort whose later
// histograms were not produced upstream).
// GATHER: the last ordering pass writes the caller's edges (position < k)
// instead of the next key/value buffers.
struct GatherOut {
  const uint32_t* cu;
  const uint32_t* cw;
  const float* cs;
  uint64_t k;
  EdgeOut* out;
  uint64_t* ctr;   // the call's counters: C_OUT_N is set, all are published to hctr
  uint64_t* hctr;  // host-mapped copy of the counters (read after the call's final event)
  const uint64_t* ts;  // the call's timing stamps, published to hctr[NCTR ..]
  // device word OR-ed with the call's flags (nlp_predict_device_async: a redo
  // needed by any call of a batch shows at nlp_sync; the calls of one handle
  // run in stream order, so a plain read-modify-write is enough)
  uint64_t* sticky = nullptr;
};

// Exclusive scan of one value per digit (threads 0-255, 0 elsewhere) over the
// 256 digits, by all threads of an OS_NT workgroup; also returns the total.
__device__ __forceinline__ uint32_t os_digit_scan(uint32_t x, uint32_t* s_w, uint64_t* total) {
  const int lane = lane_id(), wv = wave_id();
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63 && wv < 4) s_w[wv] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    pre += w < wv ? s_w[w] : 0u;
    tot += s_w[w];
  }
  *total = tot;
  __syncthreads();
  return pre + inc - x;
}

enum { GAP_NONE = 0, GAP_SEGMENTS = 1, GAP_BUCKETS = 2 };
// Counted passes (k_sp_cpass): at most CP_MAXT tiles of OS2_TILE keys, so the
// per-tile digit counts of a pass fit one LDS matrix of u16 pairs.
constexpr int CP_MAXT = 128;
constexpr int CP_THW = CP_MAXT * 256 / 2;
// Exclusive scan of one value per thread over an OS_NT workgroup (s_w: OS_NW
// words); also returns the total.
__device__ __forceinline__ uint32_t os_block_scan(uint32_t x, uint32_t* s_w, uint64_t* total) {
  const int lane = lane_id(), wv = wave_id();
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < OS_NW; ++w) {
    pre += w < wv ? s_w[w] : 0u;
    tot += s_w[w];
  }
  *total = tot;
  __syncthreads();
  return pre + inc - x;
}

template <typename K, int IPT = OS2_IPT, bool GATHER = false, bool NEXT_HIST = false, int GAPPED = GAP_NONE, int DB = 8>
__global__ __launch_bounds__(OS_NT) void k_sp_pass(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                   K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                   const uint64_t* __restrict__ d_n, int shift,
                                                   const uint32_t* __restrict__ ghist, uint32_t* __restrict__ desc,
                                                   uint32_t* __restrict__ tick, uint32_t* __restrict__ err,
                                                   uint64_t* __restrict__ stamp, GatherOut go,
                                                   uint32_t* __restrict__ nhist = nullptr,
                                                   const uint32_t* __restrict__ seg_cnt = nullptr,
                                                   uint64_t* __restrict__ tot_out = nullptr,
                                                   const uint64_t* __restrict__ abort_flags = nullptr,
                                                   uint32_t nseg = 0, int seglog = 0,
                                                   uint64_t* __restrict__ end_mark = nullptr,
                                                   uint32_t* __restrict__ clean_desc = nullptr) {
  constexpr int WT = 64 * IPT;
  constexpr int TILE = OS_NT * IPT;
  using PD = PassDigits<DB>;
  constexpr int NB = PD::NB, ND = PD::ND, NHD = PD::NHD;
  constexpr uint32_t DMASK = NB - 1;
  using CT = typename PD::CT;
  static_assert(!GAPPED || (RU_SEG % 64 == 0), "a wave substep must lie in one segment");
  static_assert(DB == 8 || sizeof(K) == 4, "11-bit digits: 32-bit keys");
  __shared__ CT s_wcnt[OS_NW][NB];
  __shared__ uint32_t s_base[NB];
  __shared__ uint32_t s_dbase[DB == 8 ? 1 : NB];
  __shared__ uint32_t s_nh[NEXT_HIST ? NHD : 1][NEXT_HIST ? NB : 1];
  __shared__ uint32_t s_w[OS_NW];
  __shared__ uint32_t s_tile[2];
  __shared__ uint32_t s_pre[GAPPED == GAP_BUCKETS ? DX_MAXB + 1 : 1];
  __shared__ uint32_t s_w16[GAPPED == GAP_BUCKETS ? OS_NW : 1];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  ts_mark_end(end_mark);  // the end of the kernel before (the hot kernel's, for the first ordering pass)
  // abort_flags: a range of the grouping raised F_TOOBIG, so the input holds
  // stale slots and the call is redone -- order nothing (and count 0 candidates)
  const bool abort = abort_flags && (*abort_flags & F_TOOBIG);
  uint64_t n = abort ? 0 : *d_n;
  if (GAPPED == GAP_BUCKETS) {
    // GAP_BUCKETS: segment b holds seg_cnt[b] keys at slots [b 2^seglog, ...);
    // dense index j lies in the segment with s_pre[b] <= j < s_pre[b + 1]
    constexpr uint32_t PER = (DX_MAXB + OS_NT - 1) / OS_NT;
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const uint32_t b = (uint32_t)t * PER + q;
      c[q] = b < nseg ? seg_cnt[b] : 0u;
      sum += c[q];
    }
    uint64_t tot;
    uint32_t run = os_block_scan(sum, s_w16, &tot);  // (GAP_BUCKETS prologue)
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const uint32_t b = (uint32_t)t * PER + q;
      if (b < nseg) s_pre[b] = run;
      run += c[q];
    }
    if (t == 0) s_pre[nseg] = (uint32_t)tot;
    __syncthreads();
    n = tot;
  }
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  if (GAPPED && abort && tot_out && blockIdx.x == 0 && t == 0) *tot_out = 0;
  // GATHER: every counter is final by now; they are published by the workgroup
  // of the last tile after its scatter (or by workgroup 0 when there is no tile)
  auto publish = [&]() {
    if (GATHER && t < NCTR) {
      const uint64_t m = n < go.k ? n : go.k;
      if (t == C_OUT_N) go.ctr[C_OUT_N] = m;
      // host-coherent memory; the call's final event (a system-scope release)
      // orders these stores before the host reads them
      if (go.hctr) go.hctr[t] = t == C_OUT_N ? m : go.ctr[t];
      if (go.hctr && go.ts && t < TS_END) go.hctr[NCTR + t] = go.ts[t];
      if (go.hctr && t == 0) go.hctr[NCTR + TS_END] = __builtin_amdgcn_s_memrealtime();  // the last tile: ~the end
      if (go.sticky && t == C_FLAGS) *go.sticky |= go.ctr[C_FLAGS];
    }
  };
  if (GATHER && ntiles == 0 && blockIdx.x == 0) publish();
  if (blockIdx.x >= ntiles) return;  // only as many claimants as tiles
  sp_stamp(stamp, true, 7);           // entry (diagnostics: ticket + digit bases until phase 0)
  if (t == 0) s_tile[0] = atomicAdd(tick, 1u);
  if (NEXT_HIST)
    for (int i = t; i < NHD * NB; i += OS_NT) (&s_nh[0][0])[i] = 0;
  uint64_t tot;
  uint32_t dbase = 0;  // DB == 8: digit t's base (t < 256); else s_dbase
  if (DB == 8) {
    dbase = os_digit_scan(t < RS_BINS ? hist_total(ghist, t) : 0u, s_w, &tot);  // syncs
  } else {  // thread t: digits [ND t, ND t + ND)
    uint32_t c[ND], sum = 0;
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      c[q] = hist_total_db<DB>(ghist, (uint32_t)t * ND + q);
      sum += c[q];
    }
    uint32_t run = os_block_scan(sum, s_w, &tot);  // syncs
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      s_dbase[t * ND + q] = run;
      run += c[q];
    }
  }
  const uint64_t lt = lane_mask_lt();
  bool first = true;
  for (int par = 0;; par ^= 1) {
    const uint64_t tile = s_tile[par];
    if (tile >= ntiles) break;
    if (GAPPED && tile == 0 && t == 0 && tot_out) *tot_out = tot;
    sp_stamp(stamp, first, 0);
    for (int i = t; i < OS_NW * NB * (int)sizeof(CT) / 4; i += OS_NT) ((uint32_t*)&s_wcnt[0][0])[i] = 0;
    __syncthreads();
    if (t == 0) s_tile[par ^ 1] = atomicAdd(tick, 1u);  // claim the next tile meanwhile
    const uint64_t b0 = tile * TILE + (uint64_t)wv * WT + lane;
    K k[IPT];
    uint32_t v[IPT], dg[IPT], rk[IPT];
    bool ok[IPT];
    uint32_t seg_lo = 0;  // GAP_BUCKETS: the segment of the wave's first index
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint64_t j = b0 + (uint64_t)i * 64;
      ok[i] = j < n;
      if (GAPPED == GAP_SEGMENTS && ok[i]) ok[i] = (uint32_t)(j % RU_SEG) < seg_cnt[j / RU_SEG];
      uint64_t sj = j;
      if (GAPPED == GAP_BUCKETS) {
        // the segment holding dense index j (last b with s_pre[b] <= j): one
        // search for the wave's first index of the first substep (uniform),
        // then short walks -- consecutive indices cross few segment boundaries
        if (i == 0) {
          const uint32_t j0 = (uint32_t)(b0 - lane);
          uint32_t hi = nseg;  // s_pre[seg_lo] <= j0 < s_pre[hi]
          seg_lo = 0;
          while (hi - seg_lo > 1) {
            const uint32_t mid = (seg_lo + hi) >> 1;
            if (s_pre[mid] <= j0) seg_lo = mid;
            else hi = mid;
          }
        }
        if (ok[i]) {
          uint32_t lo = seg_lo;
          while (s_pre[lo + 1] <= (uint32_t)j) ++lo;
          sj = ((uint64_t)lo << seglog) + ((uint32_t)j - s_pre[lo]);
        }
      }
      k[i] = ok[i] ? kin[sj] : (K)0;
      v[i] = ok[i] && vin ? vin[sj] : 0u;  // vin null: keys only
    }
    EdgeOut eo[GATHER ? IPT : 1];
    if (GATHER) {  // the output columns are fetched now, in flight during ranking and look-back
#pragma unroll
      for (int i = 0; i < IPT; ++i)
        if (ok[i]) eo[i] = EdgeOut{go.cu[v[i]], go.cw[v[i]], go.cs[v[i]]};
    }
    sp_stamp(stamp, first, 1);
    // wave ranks: ballot multisplit + the wave's running digit counts
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t d = (uint32_t)(k[i] >> shift) & DMASK;
      dg[i] = d;
      uint64_t peers = __ballot(ok[i]);
#pragma unroll
      for (int b = 0; b < DB; ++b) {
        const uint64_t bb = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bb : ~bb;
      }
      const uint32_t before = ok[i] ? s_wcnt[wv][d] : 0u;
      rk[i] = before + (uint32_t)__popcll(peers & lt);
      wave_lds_sync();
      if (ok[i] && (peers & lt) == 0) s_wcnt[wv][d] = (CT)(before + (uint32_t)__popcll(peers));
      wave_lds_sync();
    }
    __syncthreads();
    sp_stamp(stamp, first, 2);
    // thread t owns digits t, t + OS_NT, ..: wave prefix, aggregate, look-back, inclusive prefix
    if (t < NB) {
      uint32_t dd[ND], run[ND], excl[ND];
#pragma unroll
      for (int q = 0; q < ND; ++q) {
        dd[q] = (uint32_t)t + (uint32_t)q * OS_NT;
        run[q] = 0;
#pragma unroll
        for (int w = 0; w < OS_NW; ++w) {
          const uint32_t c = s_wcnt[w][dd[q]];
          s_wcnt[w][dd[q]] = (CT)run[q];
          run[q] += c;
        }
        st_u32(desc + tile * NB + dd[q], (tile == 0 ? OS_PFX : OS_AGG) | run[q]);
      }
      os_lookback<ND, PD::LBW>(desc, (uint32_t)NB, tile, dd, excl, err);
#pragma unroll
      for (int q = 0; q < ND; ++q) {
        if (tile != 0) st_u32(desc + tile * NB + dd[q], OS_PFX | (excl[q] + run[q]));
        s_base[dd[q]] = (DB == 8 ? dbase : s_dbase[dd[q]]) + excl[q];
      }
    }
    __syncthreads();
    sp_stamp(stamp, first, 3);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      if (ok[i]) {
        const uint64_t pos = (uint64_t)s_base[dg[i]] + s_wcnt[wv][dg[i]] + rk[i];
        if (GATHER) {
          if (pos < go.k) go.out[pos] = eo[i];
        } else {
          kout[pos] = k[i];
          if (vout) vout[pos] = v[i];
        }
        if (NEXT_HIST) {
#pragma unroll
          for (int dd = 0; dd < NHD; ++dd) atomicAdd(&s_nh[dd][(uint32_t)(k[i] >> (DB * dd + DB)) & DMASK], 1u);
        }
      }
    }
    // clean_desc: the previous pass's descriptors (same tile count), finished
    // with -- row `tile` back to zero for the next call (no zeroing pass)
    for (int i = t; clean_desc && i < NB; i += OS_NT) st_u32(&clean_desc[tile * NB + i], 0u);
    __syncthreads();
    sp_stamp(stamp, first, 4);
    if (GATHER && tile == ntiles - 1) publish();
    first = false;
  }
  if (NEXT_HIST) {
    uint32_t* hc = hist_copy_db<DB>(nhist);
    for (int i = t; i < NHD * NB; i += OS_NT) {
      const uint32_t c = s_nh[i / NB][i % NB];
      if (c) atomicAdd(&hc[i], c);
    }
  }
}

// ---------------------------------------------------------------- counted passes
// The fused path's four ordering passes without look-back (round 2).  Each
// pass reads, instead of a look-back, a count matrix that the kernel before it
// produced: m[tile][digit] = the keys of input tile `tile` with digit `digit`.
// A tile's base for digit d is (sum over d' < d of the digit totals) + (digit
// d's counts in the tiles before it): tiles share no descriptor, no ticket and
// wait on nothing, so any grid size and dispatch order works.
//
//   k_sp_grouprun   counts digit 0 per bucket group into m0
//   k_sp_cpass0     tile = 4096 consecutive keys of the concatenated buckets
//                   (their slots, in bucket order = (u, w) order); counts digit
//                   1 per output tile (m1)
//   k_sp_cpass x3   tile = OS2_TILE consecutive keys; passes 1 and 2 count the
//                   next digit per output tile (m2, m3); pass 3 writes the
//                   caller's edges (GATHER) and publishes the counters
//
// The keys travel with their payload (u << 32 | w, score bits), so the last
// pass writes the edges without a random gather of candidate columns.  The
// per-output-tile counts are kept in LDS as u16 pairs (a bin holds at most
// OS2_TILE keys) and flushed with one atomic per non-zero bin, which bounds the
// output to CP_MAXT tiles: beyond it k_sp_cpass0 raises F_CPASS, every later
// pass returns at once, and the host redoes the call with look-back passes.
// Cleaning: pass 1 zeroes m0, pass 2 m1, pass 3 m2 (row = its workgroup,
// before any early exit); m3 -- read by every tile of the last pass -- is
// zeroed by pass 1 of the next call (all CP_MAXT rows), before pass 2 counts
// into it.

// Digit bases of tile `tile` of `ntiles` from the count matrix m: s_base[d] =
// (totals of the digits below d) + (digit d in tiles < tile); returns the key
// total n.  All threads of an OS_NT workgroup; ends with a barrier.
// m: packed u16 pairs (bin 2i in the low half of word i) -- the matrices the
// passes count into; a bin holds at most OS2_TILE keys.
__device__ __forceinline__ uint64_t cp_bases(const uint32_t* __restrict__ m32, uint32_t ntiles, uint32_t tile,
                                             uint32_t (&s_part)[2][OS_NT / RS_BINS][RS_BINS], uint32_t* s_base,
                                             uint32_t* s_w) {
  constexpr uint32_t Q = OS_NT / RS_BINS;
  const int t = threadIdx.x;
  const uint16_t* m = (const uint16_t*)m32;
  {  // thread t: digit t % 256 over the tiles r = t / 256 (mod Q), all loads in one round trip
    constexpr int R = CP_MAXT / Q;
    const uint32_t d = (uint32_t)t % RS_BINS, q = (uint32_t)t / RS_BINS;
    uint32_t c[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint32_t r = q + (uint32_t)i * Q;
      c[i] = m[(r < ntiles ? r : 0u) * RS_BINS + d];  // ntiles >= 1
    }
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint32_t r = q + (uint32_t)i * Q;
      total += r < ntiles ? c[i] : 0u;
      before += r < tile ? c[i] : 0u;
    }
    s_part[0][q][d] = before;
    s_part[1][q][d] = total;
  }
  __syncthreads();
  uint32_t before = 0, total = 0;
  if (t < RS_BINS) {
#pragma unroll
    for (uint32_t q = 0; q < Q; ++q) {
      before += s_part[0][q][t];
      total += s_part[1][q][t];
    }
  }
  uint64_t n;
  const uint32_t dbase = os_digit_scan(total, s_w, &n);  // syncs
  if (t < RS_BINS) s_base[t] = dbase + before;
  __syncthreads();
  return n;
}

// Ballot-multisplit ranks of IPT keys per lane (wave wv owns 64 IPT
// consecutive keys): rk = rank among the wave's earlier keys of the same digit;
// s_wcnt[wv][d] = the wave's count of digit d (zeroed by the caller).
template <int IPT>
__device__ __forceinline__ void cp_rank(const uint32_t (&k)[IPT], const bool (&ok)[IPT], int shift,
                                        uint32_t (&dg)[IPT], uint32_t (&rk)[IPT], uint32_t (*s_wcnt)[RS_BINS]) {
  const int wv = wave_id();
  const uint64_t lt = lane_mask_lt();
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const uint32_t d = (k[i] >> shift) & 255u;
    dg[i] = d;
    uint64_t peers = __ballot(ok[i]);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t pre = ok[i] ? s_wcnt[wv][d] : 0u;
    rk[i] = pre + (uint32_t)__popcll(peers & lt);
    wave_lds_sync();
    if (ok[i] && (peers & lt) == 0) s_wcnt[wv][d] = pre + (uint32_t)__popcll(peers);
    wave_lds_sync();
  }
}

// Wave prefixes of digit t (t < 256): s_wcnt[w][t] <- keys of digit t in
// waves < w; returns the tile's count of digit t.
__device__ __forceinline__ uint32_t cp_wave_prefix(uint32_t (*s_wcnt)[RS_BINS], int t) {
  uint32_t run = 0;
#pragma unroll
  for (int w = 0; w < OS_NW; ++w) {
    const uint32_t c = s_wcnt[w][t];
    s_wcnt[w][t] = run;
    run += c;
  }
  return run;
}

// Count of (output tile, next digit) of one placed key, into the LDS u16 pairs.
__device__ __forceinline__ void cp_count_next(uint32_t* s_th, uint32_t pos, uint32_t key, int nshift) {
  const uint32_t bin = (pos / OS2_TILE) * RS_BINS + ((key >> nshift) & 255u);
  atomicAdd(&s_th[bin >> 1], 1u << ((bin & 1u) * 16));  // a bin holds <= OS2_TILE keys: no carry
}
// The output matrix keeps the LDS layout (u16 pairs): one atomic per non-zero
// pair, no carry between the halves (a bin holds at most OS2_TILE keys).
__device__ __forceinline__ void cp_flush_next(const uint32_t* s_th, uint32_t ntiles, uint32_t* __restrict__ hout) {
  for (uint32_t i = threadIdx.x; i < ntiles * (RS_BINS / 2); i += OS_NT) {
    const uint32_t c = s_th[i];
    if (c) atomicAdd(&hout[i], c);
  }
}

// Pass 0: tile = OS2_TILE consecutive keys of the concatenated buckets (dense
// position P = bucket prefix + slot), gridDim >= tiles.  m0 holds digit 0 per
// bucket GROUP (G consecutive buckets, counted by k_sp_grouprun), so the digit
// bases of tile j at P_j = j OS2_TILE are (totals of the lower digits) + (m0
// rows of the groups before P_j's group) + (the digit's count among that
// group's keys before P_j, counted here from the keys themselves).  Every tile
// holds exactly OS2_TILE keys (the last one fewer): no imbalance between tiles
// whatever the bucket sizes.  The candidate count (the matrix total) goes to
// ctr[C_C].
__global__ __launch_bounds__(OS_NT) void k_sp_cpass0(const uint32_t* __restrict__ okey, const uint32_t* __restrict__ cu,
                                                     const uint32_t* __restrict__ cw, const float* __restrict__ cs,
                                                     const uint32_t* __restrict__ kcnt, uint32_t nb, uint32_t G,
                                                     uint32_t ngroups, int caplog, const uint32_t* __restrict__ m0,
                                                     uint32_t* __restrict__ m1, uint32_t* __restrict__ kout,
                                                     uint64_t* __restrict__ uwout, uint32_t* __restrict__ sout,
                                                     uint64_t* __restrict__ ctr, uint64_t* __restrict__ end_mark,
                                                     uint64_t* __restrict__ stamp) {
  constexpr int IPT = OS2_IPT, WT = 64 * IPT, TILE = OS2_TILE;
  constexpr uint32_t Q = OS_NT / RS_BINS, R = CP_MAXT / Q, PER = DX_MAXB / OS_NT;
  __shared__ uint32_t s_wcnt[OS_NW][RS_BINS];
  __shared__ uint32_t s_pre[DX_MAXB + 1];  // exclusive prefix of the bucket counts
  __shared__ uint32_t s_part[2][Q][RS_BINS];
  __shared__ uint32_t s_lead[RS_BINS];     // digit counts of P_j's group before P_j
  __shared__ uint32_t s_base[RS_BINS];
  __shared__ uint32_t s_w[OS_NW];
  __shared__ uint32_t s_th[CP_THW];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint32_t tile = blockIdx.x, P = tile * TILE;
  ts_mark_end(end_mark);  // the end of the kernel before (the hot kernel)
  sp_stamp(stamp, true, 7);
  // the m0 rows (all in flight while the bucket prefix is formed)
  const uint32_t d = (uint32_t)t % RS_BINS, q = (uint32_t)t / RS_BINS;
  uint32_t c[R];
#pragma unroll
  for (uint32_t i = 0; i < R; ++i) {
    const uint32_t r = q + i * Q;
    c[i] = m0[(r < ngroups ? r : 0u) * RS_BINS + d];
  }
  {  // bucket prefix: thread t sums buckets [PER t, PER t + PER)
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
      const uint32_t b = (uint32_t)t * PER + i;
      v[i] = b < nb ? kcnt[b] : 0u;
      sum += v[i];
    }
    uint64_t tot;
    uint32_t run = os_block_scan(sum, s_w, &tot);  // syncs
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
      const uint32_t b = (uint32_t)t * PER + i;
      if (b < nb) s_pre[b] = run;
      run += v[i];
    }
    if (t == 0) s_pre[nb] = (uint32_t)tot;
    if (t < RS_BINS) s_lead[t] = 0;
  }
  for (int i = t; i < OS_NW * RS_BINS; i += OS_NT) (&s_wcnt[0][0])[i] = 0;
  __syncthreads();
  const uint32_t n = s_pre[nb];
  if (tile == 0 && t == 0) ctr[C_C] = n;
  const uint32_t ntiles = (n + TILE - 1) / TILE;
  if (ntiles > (uint32_t)CP_MAXT) {  // beyond the counted passes: redone with look-back passes
    if (tile == 0 && t == 0) atomicOr((unsigned long long*)&ctr[C_FLAGS], (unsigned long long)F_CPASS);
    return;
  }
  if (tile >= ntiles) return;
  // bucket of a dense position: last b with s_pre[b] <= x (a uniform search)
  auto bucket_of = [&](uint32_t x) {
    uint32_t lo = 0, hi = nb;  // s_pre[lo] <= x < s_pre[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_pre[mid] <= x) lo = mid;
      else hi = mid;
    }
    return lo;
  };
  const uint32_t bj = bucket_of(P), gj = bj / G, gp = s_pre[gj * G];  // P_j's group and its dense start
  {
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t i = 0; i < R; ++i) {
      const uint32_t r = q + i * Q;
      total += r < ngroups ? c[i] : 0u;
      before += r < gj ? c[i] : 0u;
    }
    s_part[0][q][d] = before;
    s_part[1][q][d] = total;
  }
  for (uint32_t i = t; i < ntiles * (RS_BINS / 2); i += OS_NT) s_th[i] = 0;
  // the tile's keys and payload: wave wv's keys from one search, then short walks
  uint32_t k[IPT], uu[IPT], ww[IPT], ss[IPT], dg[IPT], rk[IPT];
  bool ok[IPT];
  {
    const uint32_t j0 = P + (uint32_t)wv * WT;
    uint32_t b = bucket_of(j0 < n ? j0 : 0u);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint32_t j = j0 + (uint32_t)i * 64 + (uint32_t)lane;
      ok[i] = j < n && j < P + TILE;
      if (ok[i]) {
        while (s_pre[b + 1] <= j) ++b;
        const uint64_t slot = ((uint64_t)b << caplog) + (j - s_pre[b]);
        k[i] = okey[slot];
        uu[i] = cu[slot];
        ww[i] = cw[slot];
        ss[i] = __float_as_uint(cs[slot]);
      } else {
        k[i] = uu[i] = ww[i] = ss[i] = 0u;
      }
    }
  }
  {  // the digit counts of the group's keys in [gp, P) (in LDS), LP keys per thread per round with all
     // loads in flight together
    constexpr int LP = 8;
    for (uint32_t x0 = gp; x0 < P; x0 += LP * OS_NT) {
      uint32_t kk[LP];
      uint32_t b = bucket_of(x0 + (uint32_t)t < P ? x0 + (uint32_t)t : x0);
#pragma unroll
      for (int i = 0; i < LP; ++i) {
        const uint32_t x = x0 + (uint32_t)t + (uint32_t)i * OS_NT;
        kk[i] = 0u;
        if (x < P) {
          while (s_pre[b + 1] <= x) ++b;
          kk[i] = okey[((uint64_t)b << caplog) + (x - s_pre[b])];
        }
      }
#pragma unroll
      for (int i = 0; i < LP; ++i)
        if (x0 + (uint32_t)t + (uint32_t)i * OS_NT < P) atomicAdd(&s_lead[kk[i] & 255u], 1u);
    }
  }
  __syncthreads();  // s_part, s_lead
  {
    uint32_t before = 0, total = 0;
    if (t < RS_BINS) {
#pragma unroll
      for (uint32_t i = 0; i < Q; ++i) {
        before += s_part[0][i][t];
        total += s_part[1][i][t];
      }
      before += s_lead[t];
    }
    uint64_t tot;
    const uint32_t dbase = os_digit_scan(total, s_w, &tot);  // syncs
    if (t < RS_BINS) s_base[t] = dbase + before;
  }
  sp_stamp(stamp, true, 0);
  cp_rank<IPT>(k, ok, 0, dg, rk, s_wcnt);
  __syncthreads();
  sp_stamp(stamp, true, 2);
  if (t < RS_BINS) cp_wave_prefix(s_wcnt, t);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    if (ok[i]) {
      const uint32_t pos = s_base[dg[i]] + s_wcnt[wv][dg[i]] + rk[i];
      kout[pos] = k[i];
      uwout[pos] = ((uint64_t)uu[i] << 32) | ww[i];
      sout[pos] = ss[i];
      cp_count_next(s_th, pos, k[i], 8);
    }
  }
  __syncthreads();
  cp_flush_next(s_th, ntiles, m1);
  sp_stamp(stamp, true, 4);
}

// Passes 1-3: tile = blockIdx (OS2_TILE consecutive keys).  NEXT: count the
// next digit per output tile into hout.  clean: row blockIdx (< clean_rows,
// 0 = this pass's tile count) of a finished pass's matrix back to zero.
// GATHER (the last pass): the caller's edges at positions below go.k;
// workgroup 0 publishes the counters and stamps (the call's counters are final),
// the last tile the end stamp.
template <bool NEXT, bool GATHER = false>
__global__ __launch_bounds__(OS_NT) void k_sp_cpass(const uint32_t* __restrict__ kin, const uint64_t* __restrict__ uwin,
                                                    const uint32_t* __restrict__ sin, uint32_t* __restrict__ kout,
                                                    uint64_t* __restrict__ uwout, uint32_t* __restrict__ sout,
                                                    const uint64_t* __restrict__ d_n, int shift,
                                                    const uint32_t* __restrict__ hin, uint32_t* __restrict__ hout,
                                                    uint32_t* __restrict__ clean, uint32_t clean_rows,
                                                    uint32_t clean_words, uint64_t* __restrict__ stamp, GatherOut go,
                                                    uint32_t* __restrict__ clean_all = nullptr) {
  constexpr int IPT = OS2_IPT, WT = 64 * IPT, TILE = OS2_TILE;
  __shared__ uint32_t s_wcnt[OS_NW][RS_BINS];
  __shared__ uint32_t s_part[2][OS_NT / RS_BINS][RS_BINS];
  __shared__ uint32_t s_base[RS_BINS];
  __shared__ uint32_t s_w[OS_NW];
  __shared__ uint32_t s_th[NEXT ? CP_THW : 1];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = *d_n;
  const uint32_t ntiles = (uint32_t)((n + TILE - 1) / TILE);
  const uint32_t tile = blockIdx.x;
  if (clean && tile < (clean_rows ? clean_rows : ntiles))  // rows of clean_words words
    for (uint32_t i = t; i < clean_words; i += OS_NT) clean[(uint64_t)tile * clean_words + i] = 0u;
  if (clean_all)  // every packed row (gridDim = CP_MAXT): a matrix of the previous call, whatever its tile count
    for (int i = t; i < RS_BINS / 2; i += OS_NT) clean_all[(uint64_t)tile * (RS_BINS / 2) + i] = 0u;
  if (GATHER && tile == 0 && t < NCTR) {  // every counter is final: published now (also with no tile)
    const uint64_t m = n < go.k ? n : go.k;
    if (t == C_OUT_N) go.ctr[C_OUT_N] = m;
    if (go.sticky && t == C_FLAGS) *go.sticky |= go.ctr[C_FLAGS];
    if (go.hctr) {
      go.hctr[t] = t == C_OUT_N ? m : go.ctr[t];
      if (go.ts && t < TS_END) go.hctr[NCTR + t] = go.ts[t];
      if (t == 0 && (ntiles == 0 || ntiles > (uint32_t)CP_MAXT))
        go.hctr[NCTR + TS_END] = __builtin_amdgcn_s_memrealtime();
      __threadfence_system();
    }
  }
  if (tile >= ntiles || ntiles > (uint32_t)CP_MAXT) return;  // beyond CP_MAXT: F_CPASS is raised, the call redone
  sp_stamp(stamp, true, 7);
  const uint64_t b0 = (uint64_t)tile * TILE + (uint64_t)wv * WT + lane;
  uint32_t k[IPT], ss[IPT], dg[IPT], rk[IPT];
  uint64_t uw[IPT];
  bool ok[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) {  // the tile's keys, in flight during the matrix reads
    const uint64_t j = b0 + (uint64_t)i * 64;
    ok[i] = j < n;
    k[i] = ok[i] ? kin[j] : 0u;
    uw[i] = ok[i] ? uwin[j] : 0ull;
    ss[i] = ok[i] ? sin[j] : 0u;
  }
  for (int i = t; i < OS_NW * RS_BINS; i += OS_NT) (&s_wcnt[0][0])[i] = 0;
  if (NEXT)
    for (uint32_t i = t; i < ntiles * (RS_BINS / 2); i += OS_NT) s_th[i] = 0;
  cp_bases(hin, ntiles, tile, s_part, s_base, s_w);  // syncs
  sp_stamp(stamp, true, 0);
  cp_rank<IPT>(k, ok, shift, dg, rk, s_wcnt);
  __syncthreads();
  sp_stamp(stamp, true, 2);
  if (t < RS_BINS) cp_wave_prefix(s_wcnt, t);
  __syncthreads();
  sp_stamp(stamp, true, 3);
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    if (ok[i]) {
      const uint32_t pos = s_base[dg[i]] + s_wcnt[wv][dg[i]] + rk[i];
      if (GATHER) {
        if (pos < go.k) go.out[pos] = EdgeOut{(uint32_t)(uw[i] >> 32), (uint32_t)uw[i], __uint_as_float(ss[i])};
      } else {
        kout[pos] = k[i];
        uwout[pos] = uw[i];
        sout[pos] = ss[i];
      }
      if (NEXT) cp_count_next(s_th, pos, k[i], shift + 8);
    }
  }
  if (NEXT) {
    __syncthreads();
    cp_flush_next(s_th, ntiles, hout);
  }
  sp_stamp(stamp, true, 4);
  // the call's end: the last tile's exit (approximately the last workgroup's)
  if (GATHER && go.hctr && tile == ntiles - 1 && t == 0) go.hctr[NCTR + TS_END] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------- small calls: ordering by rank
// When the candidates of a fused call fit SO_MAX keys (the LHub-4 calls of the
// large configs: C4 predicts ~1e4 links), the four counted passes -- four
// launches, each waiting for the previous one's keys to land -- are replaced
// by ONE launch that ranks every candidate directly.  Every workgroup loads
// all n order keys (thread t: positions i OS_NT + t of the concatenated
// buckets, (u, w) order) and groups them in LDS by bin = (key - kmin) >> sh,
// with sh the smallest shift that leaves 2^14 bins over the call's key range;
// the rest of the key and the position fit one 32-bit composite
// ((key - kmin) mod 2^sh) << 14 | position, unique within a bin.  The rank of
// candidate e in the stable sort by key (score descending, then (u, w)
// ascending -- the canonical order) is then
//   rank(e) = start(bin(e)) + #{j in bin(e) : composite_j < composite_e},
// one comparison per member of its own bin instead of per candidate (the
// n^2 / 64 comparisons of counting against every key were the whole cost).
// Workgroup g ranks the positions [g Q, (g + 1) Q), Q = ceil(n / gridDim), on
// the threads that loaded them (key, bin and slot already in registers) and
// gathers each one below k to the caller's edges.  More than SO_MAX
// candidates raise F_SMALL and the host redoes the call with the counted
// passes.  Workgroup 0 publishes the counters like the last counted pass.
constexpr uint32_t SO_MAX = 16384;  // candidates at most (positions: 14 bits)
constexpr int SR_BITS = 14;         // bins over the key range
constexpr uint32_t SR_GRID = 256;   // one workgroup per CU (LDS: ~144 KiB)

__global__ __launch_bounds__(OS_NT) void k_sp_order_rank(const uint32_t* __restrict__ okey,
                                                         const uint32_t* __restrict__ cu,
                                                         const uint32_t* __restrict__ cw,
                                                         const float* __restrict__ cs,
                                                         const uint32_t* __restrict__ kcnt, uint32_t nb, int caplog,
                                                         GatherOut go, uint64_t* __restrict__ end_mark,
                                                         uint64_t* __restrict__ stamp = nullptr) {
  constexpr uint32_t PER = (DX_MAXB + OS_NT - 1) / OS_NT;
  constexpr int LD = (int)(SO_MAX / OS_NT);  // positions per thread
  constexpr uint32_t NBIN = 1u << SR_BITS;
  constexpr int BPT = (int)(NBIN / OS_NT);   // bins per thread in the scan
  static_assert(SO_MAX <= (1u << SR_BITS) && BPT % 4 == 0, "order_rank layout");
  __shared__ __attribute__((aligned(16))) uint32_t s_bin[NBIN];  // counts, then starts, then ends
  __shared__ __attribute__((aligned(16))) uint32_t s_list[SO_MAX + 16];  // the composites, grouped by bin
  __shared__ uint32_t s_pre[DX_MAXB + 1];
  __shared__ uint32_t s_w[OS_NW];
  __shared__ uint32_t s_mm[2];
  const int t = threadIdx.x;
  ts_mark_end(end_mark);  // the end of the kernel before (the hot kernel)
  sp_stamp(stamp, true, 7);
  if (t == 0) { s_mm[0] = 0xffffffffu; s_mm[1] = 0u; }
  {  // bucket prefix: thread t sums buckets [PER t, PER t + PER)
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
      const uint32_t b = (uint32_t)t * PER + i;
      v[i] = b < nb ? kcnt[b] : 0u;
      sum += v[i];
    }
    uint64_t tot;
    uint32_t run = os_block_scan(sum, s_w, &tot);  // syncs
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
      const uint32_t b = (uint32_t)t * PER + i;
      if (b < nb) s_pre[b] = run;
      run += v[i];
    }
    if (t == 0) s_pre[nb] = (uint32_t)tot;
  }
  __syncthreads();
  const uint32_t n = s_pre[nb];
  uint64_t* ctr = go.ctr;
  const bool fits = n <= SO_MAX;
  const uint64_t m = fits ? (n < go.k ? (uint64_t)n : go.k) : 0ull;
  const uint32_t Q = (n + gridDim.x - 1) / gridDim.x;
  const uint32_t q0 = blockIdx.x * Q;
  sp_stamp(stamp, true, 0);
  if (fits && q0 < n) {
    // keys in position order: thread t owns positions [LD t, LD t + LD) (one
    // search for its first bucket, then a walk over the bucket starts), stores
    // them in LDS (s_list, free until the scatter), then reads back its
    // strided positions i OS_NT + t
    {
      const uint32_t p0 = (uint32_t)t * LD;
      uint32_t b = 0, hi = nb;  // last b with s_pre[b] <= p0
      while (hi - b > 1) {
        const uint32_t mid = (b + hi) >> 1;
        if (s_pre[mid] <= p0) b = mid; else hi = mid;
      }
      uint32_t sl[LD], kb[LD];
#pragma unroll
      for (int i = 0; i < LD; ++i) {
        const uint32_t p = p0 + (uint32_t)i;
        while (b + 1 < nb && s_pre[b + 1] <= p) ++b;
        sl[i] = p < n ? (b << caplog) + (p - s_pre[b]) : 0u;
      }
#pragma unroll
      for (int i = 0; i < LD; ++i) kb[i] = okey[sl[i]];  // slot 0 always exists
#pragma unroll
      for (int i = 0; i < LD; ++i)
        if (p0 + (uint32_t)i < n) s_list[p0 + i] = kb[i];
    }
    __syncthreads();
    uint32_t kk[LD];
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const uint32_t j = (uint32_t)i * OS_NT + (uint32_t)t;
      kk[i] = j < n ? s_list[j] : 0u;
    }
    uint32_t kmin = 0xffffffffu, kmax = 0u;
    sp_stamp(stamp, true, 1);
#pragma unroll
    for (int i = 0; i < LD; ++i)
      if ((uint32_t)i * OS_NT + (uint32_t)t < n) {
        kmin = min(kmin, kk[i]);
        kmax = max(kmax, kk[i]);
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o, 64));
      kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
    }
    if (lane_id() == 0) {
      atomicMin(&s_mm[0], kmin);
      atomicMax(&s_mm[1], kmax);
    }
    for (uint32_t i = t; i < NBIN; i += OS_NT) s_bin[i] = 0u;
    __syncthreads();
    sp_stamp(stamp, true, 2);
    kmin = s_mm[0];
    const uint32_t span = s_mm[1] - kmin;
    const int lb = span ? 32 - __clz(span) : 0;
    const int sh = lb > SR_BITS ? lb - SR_BITS : 0;
    uint32_t bn[LD];
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      bn[i] = (kk[i] - kmin) >> sh;
      if ((uint32_t)i * OS_NT + (uint32_t)t < n) atomicAdd(&s_bin[bn[i]], 1u);
    }
    __syncthreads();
    sp_stamp(stamp, true, 3);
    {  // exclusive starts: thread t owns bins [BPT t, BPT t + BPT)
      uint32_t c[BPT], sum = 0;
      const uint4* p = reinterpret_cast<const uint4*>(s_bin + (uint32_t)t * BPT);
#pragma unroll
      for (int i = 0; i < BPT / 4; ++i) {
        const uint4 x = p[i];
        c[4 * i] = x.x; c[4 * i + 1] = x.y; c[4 * i + 2] = x.z; c[4 * i + 3] = x.w;
      }
#pragma unroll
      for (int i = 0; i < BPT; ++i) sum += c[i];
      uint64_t tot;
      uint32_t run = os_block_scan(sum, s_w, &tot);  // syncs (every read above is done)
      uint4* w = reinterpret_cast<uint4*>(s_bin + (uint32_t)t * BPT);
#pragma unroll
      for (int i = 0; i < BPT / 4; ++i) {
        uint4 x;
        x.x = run; run += c[4 * i];
        x.y = run; run += c[4 * i + 1];
        x.z = run; run += c[4 * i + 2];
        x.w = run; run += c[4 * i + 3];
        w[i] = x;
      }
    }
    __syncthreads();
    const uint32_t lowmask = sh ? (1u << sh) - 1u : 0u;
    uint32_t cp[LD];
#pragma unroll
    for (int i = 0; i < LD; ++i) {  // group: s_bin[b] advances from the start of bin b to its end
      const uint32_t j = (uint32_t)i * OS_NT + (uint32_t)t;
      cp[i] = (((kk[i] - kmin) & lowmask) << SR_BITS) | j;
      if (j < n) s_list[atomicAdd(&s_bin[bn[i]], 1u)] = cp[i];
    }
    __syncthreads();
    sp_stamp(stamp, true, 4);
#pragma unroll
    for (int i = 0; i < LD; ++i) {  // this workgroup's positions: rank within the bin, gather
      const uint32_t j = (uint32_t)i * OS_NT + (uint32_t)t;
      if (j < q0 || j >= q0 + Q || j >= n) continue;
      const uint32_t b = bn[i];
      const uint32_t bs = b ? s_bin[b - 1] : 0u, be = s_bin[b];
      uint32_t r = bs;
      for (uint32_t x = bs & ~3u; x < be; x += 16) {  // 16 members per round of LDS reads (4 x 16 B)
        uint4 q[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) q[h] = *reinterpret_cast<const uint4*>(s_list + x + 4 * h);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t y = x + 4 * h;
          r += (y >= bs && y < be && q[h].x < cp[i]) ? 1u : 0u;
          r += (y + 1 >= bs && y + 1 < be && q[h].y < cp[i]) ? 1u : 0u;
          r += (y + 2 >= bs && y + 2 < be && q[h].z < cp[i]) ? 1u : 0u;
          r += (y + 3 >= bs && y + 3 < be && q[h].w < cp[i]) ? 1u : 0u;
        }
      }
      if (r < m) {  // the bucket slot of position j (a few per workgroup: one search each)
        uint32_t lo = 0, hi = nb;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (s_pre[mid] <= j) lo = mid; else hi = mid;
        }
        const uint32_t s = (lo << caplog) + (j - s_pre[lo]);
        go.out[r] = EdgeOut{cu[s], cw[s], cs[s]};
      }
    }
  }
  sp_stamp(stamp, true, 5);
  if (blockIdx.x == 0 && t < NCTR) {  // counters: final once this call's kernels before this one are done
    uint64_t x = ctr[t];
    if (t == C_C) x = n;
    if (t == C_FLAGS && !fits) x |= F_SMALL;
    if (t == C_OUT_N) x = m;
    if (t == C_C || t == C_FLAGS || t == C_OUT_N) ctr[t] = x;
    if (go.sticky && t == C_FLAGS) *go.sticky |= x;
    {
      if (go.hctr) {
        go.hctr[t] = x;
        if (go.ts && t < TS_END) go.hctr[NCTR + t] = go.ts[t];
        if (t == 0) go.hctr[NCTR + TS_END] = __builtin_amdgcn_s_memrealtime();
        __threadfence_system();
      }
    }
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
                                                     uint32_t* __restrict__ vsorted = nullptr,
                                                     uint32_t* __restrict__ tick = nullptr) {
  __shared__ uint64_t s_k2[2][BK_CAP];
  __shared__ uint32_t s_oh[1][RS_BINS];
  __shared__ uint16_t s_p2[2][BK_CAP];
  __shared__ uint16_t s_cnt[BK_PER][BK_NW][RS_BINS];
  __shared__ uint32_t s_dig[RS_BINS];
  __shared__ uint16_t s_rs[BK_CAP + 1];  // start position of each (u, w) run
  __shared__ uint32_t s_wsum[BK_NW];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_start, s_bcnt, s_b;
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  // the fused variant compacts behind the preceding buckets (look-back): its
  // bucket ids come from an ordered ticket, so a bucket only waits on buckets
  // whose workgroups are running
  if (t == 0) s_b = tick ? atomicAdd(tick, 1u) : blockIdx.x;
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
    if (t == (int)s_b) {
      s_start = pre;
      s_bcnt = h;
    }
    __syncthreads();
  }
  const uint32_t start = s_start, c = s_bcnt, b = s_b;
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
      s_flag[r] = (!(sc <= min_score) && !f2_drop(g, ru[j], rw[j])) ? 1u : 0u;  // NaN passes
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

// ---------------------------------------------------------------- fixed-capacity buckets
// Count metrics at small wedge counts: the records go straight into 2^dbits
// buckets (the key's top dbits bits, key >> hshift) of CAP slots each -- no
// counting pass, no scan: k_sp_exbucket counts a workgroup's records per
// bucket in LDS, reserves its slots with one atomic per used bucket and
// writes them (any order: the count metrics ignore the wedge order).  A bucket
// beyond CAP raises F_TOOBIG (the host then takes the grouped path).  Then
// k_sp_grouprun, one workgroup per bucket: sort the bucket's
// keys in registers (bitonic network, E keys per thread: shuffles for partner
// distances below 64, LDS beyond), find the runs, score each (first-order
// exclusion, metric, minScore, MAXFACTOR2 -- as k_sp_runs), and write the
// candidates in (u, w) order into the bucket's own slots, counting digit 0 of
// their order keys.
constexpr int GR_NT = 256;  // k_sp_grouprun threads per bucket workgroup (default; 512 with NLP_GR_NT=512)
// Each bucket is split into EXB_SUB sub-buckets of CAP slots, workgroup w of
// k_sp_exbucket reserving in sub-bucket w % EXB_SUB: a sub-bucket's cursor sees
// 1/EXB_SUB of the workgroups (same-address atomics serialise).
constexpr uint32_t EXB_SUB = 8;

template <int SPT>  // survivors per thread: fewer workgroups contending for each bucket's cursor
__global__ __launch_bounds__(NT) void k_sp_exbucket(GraphView g, uint64_t ua, uint64_t ub, int wbits,
                                                    const uint32_t* __restrict__ surv, int hshift, int dbits,
                                                    int caplog, uint64_t* __restrict__ rkey,
                                                    uint32_t* __restrict__ bcnt, uint64_t* __restrict__ ctr,
                                                    uint64_t* __restrict__ wsum, uint64_t* __restrict__ ts,
                                                    const uint64_t* __restrict__ pack,
                                                    uint64_t* __restrict__ stamp = nullptr,
                                                    const uint64_t* __restrict__ pack_in = nullptr) {
  ts_enter(ts, TS_FIRST);
  sp_stamp(stamp, true, 0);
  __shared__ uint32_t s_h[DX_MAXB];
  __shared__ uint64_t s_red[NWAVE];
  const int t = threadIdx.x;
  const uint32_t nb = 1u << dbits, bm = nb - 1, cap = 1u << caplog;
  const uint64_t n = ctr[C_NV];
  if ((uint64_t)blockIdx.x * NT * SPT >= n) return;
  for (uint32_t i = t; i < nb; i += NT) s_h[i] = 0;
  __syncthreads();
  ExSurv x[SPT];
#pragma unroll
  for (int p = 0; p < SPT; ++p) {
    const uint64_t i = ((uint64_t)blockIdx.x * SPT + p) * NT + t;
    if (i >= n) ex_empty(g, x[p]);
    else if (pack) ex_load_packed(g, surv[i], pack[i], x[p], pack_in ? pack_in + i : nullptr);
    else ex_load(g, surv[i], x[p]);
  }
  uint64_t c = 0;
#pragma unroll
  for (int p = 0; p < SPT; ++p)
    ex_enum(g, x[p], ua, ub, [&](uint32_t u, uint32_t w) {
      atomicAdd(&s_h[(uint32_t)(ex_key(u, w, ua, wbits) >> hshift) & bm], 1u);
      ++c;
    });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane_id() == 0) s_red[wave_id()] = c;
  __syncthreads();
  if (t == 0) {
    uint64_t tot = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) tot += s_red[w];
    if (tot) atomicAdd((unsigned long long*)&wsum[blockIdx.x % WSUM_COPIES], (unsigned long long)tot);
  }
  sp_stamp(stamp, true, 1);
  const uint32_t sub = blockIdx.x % EXB_SUB;
  for (uint32_t b = t; b < nb; b += NT) {  // reserve: s_h[b] = this workgroup's first slot in its sub-bucket of b
    const uint32_t h = s_h[b];
    s_h[b] = h ? atomicAdd(&bcnt[b * EXB_SUB + sub], h) : 0u;
  }
  __syncthreads();
  sp_stamp(stamp, true, 2);
  bool over = false;
#pragma unroll
  for (int p = 0; p < SPT; ++p)
    ex_enum(g, x[p], ua, ub, [&](uint32_t u, uint32_t w) {
      const uint64_t key = ex_key(u, w, ua, wbits);
      const uint32_t b = (uint32_t)(key >> hshift) & bm;
      const uint32_t pos = atomicAdd(&s_h[b], 1u);
      if (pos < cap) rkey[((uint64_t)(b * EXB_SUB + sub) << caplog) + pos] = key;
      else over = true;
    });
  if (__ballot(over) && lane_id() == 0) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_TOOBIG);
  sp_stamp(stamp, true, 3);
}

// Ascending bitonic network over E * GR_NT keys, element i = t + r GR_NT in
// k[r].  Partners at distance j < 64 are fetched with ds_bpermute, 64 <= j <
// GR_NT through LDS, j >= GR_NT are in the same thread.  One compare-exchange
// is a 64-bit compare and two selects: keep the partner's key when it is on
// the wanted side.
template <int E, int NTH>
__device__ __forceinline__ void bitonic_sort(uint64_t (&k)[E], uint64_t* s, int t) {
  constexpr uint32_t N = (uint32_t)NTH * E;
  const int lane = t & 63;
#pragma unroll 1
  for (uint32_t size = 2; size <= N; size <<= 1) {
#pragma unroll 1
    for (uint32_t j = size >> 1; j > 0; j >>= 1) {
      if (j >= (uint32_t)NTH) {  // partner in the same thread: element r ^ (j / NTH)
        const uint32_t jr = j / NTH;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          if (((uint32_t)r & jr) == 0) {
            const uint32_t i = (uint32_t)t + (uint32_t)r * NTH;
            const bool asc = (i & size) == 0;
            const uint64_t x = k[r], y = k[r | jr];
            const bool sw = (x > y) == asc;
            k[r] = sw ? y : x;
            k[r | jr] = sw ? x : y;
          }
        }
        continue;
      }
      uint64_t o[E];
      if (j >= 64) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; ++r) s[t + r * NTH] = k[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; ++r) o[r] = s[(t ^ (int)j) + r * NTH];
      } else {
        const int idx = (lane ^ (int)j) << 2;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)(uint32_t)k[r]);
          const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)(uint32_t)(k[r] >> 32));
          o[r] = ((uint64_t)hi << 32) | lo;
        }
      }
      const bool upper = ((uint32_t)t & j) != 0;
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const uint32_t i = (uint32_t)t + (uint32_t)r * NTH;
        // keep the minimum when (ascending block) == (lower element)
        const bool keep_min = ((i & size) != 0) == upper;
        k[r] = ((k[r] > o[r]) == keep_min) ? o[r] : k[r];
      }
    }
  }
}

// the range's m <= E NTH keys, sorted, to s_key[0, m)
template <int E, int NTH>
__device__ __forceinline__ void gr_sort(const uint64_t* __restrict__ rkey, uint64_t start, uint32_t m,
                                        uint64_t* s_key, int t, const uint32_t* sub_pre = nullptr,
                                        int caplog = 0) {
  uint64_t k[E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t i = (uint32_t)t + (uint32_t)r * NTH;
    uint64_t slot = start + i;
    if (sub_pre && i < m) {  // key i of the bucket: in sub-bucket q with sub_pre[q] <= i < sub_pre[q + 1]
      uint32_t q = 0;
#pragma unroll
      for (uint32_t x = 1; x < EXB_SUB; ++x) q += sub_pre[x] <= i ? 1u : 0u;
      slot = start + ((uint64_t)q << caplog) + (i - sub_pre[q]);
    }
    k[r] = i < m ? rkey[slot] : ~0ull;
  }
  bitonic_sort<E, NTH>(k, s_key, t);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < E; ++r) s_key[t + r * NTH] = k[r];
  __syncthreads();
}

// exclusive scan over a NTH workgroup (s_w: (NTH / 64) words); *total = the sum
template <int NTH>
__device__ __forceinline__ uint32_t gr_scan(uint32_t x, uint32_t* s_w, uint32_t* total) {
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();  // s_w reuse
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < (NTH / 64); ++w) {
    pre += w < wv ? s_w[w] : 0u;
    tot += s_w[w];
  }
  *total = tot;
  return pre + inc - x;
}

// one workgroup per bucket (CAP = 2^CAPLOG slots, grid = nb).  Candidates go
// to the bucket's own slots [b CAP, b CAP + kcnt[b]) of the candidate columns,
// in (u, w) order; the first ordering pass (k_sp_pass<.., GAP_BUCKETS>) reads
// them densely through the prefix of kcnt.
template <int CAPLOG, int DB, int NTH>
__global__ __launch_bounds__(NTH) void k_sp_grouprun(GraphView g, int metric, float min_score, uint64_t ua,
                                                       int wbits, const uint64_t* __restrict__ rkey,
                                                       const uint32_t* __restrict__ bcnt,
                                                       uint32_t* __restrict__ cu, uint32_t* __restrict__ cw,
                                                       float* __restrict__ cs, uint32_t* __restrict__ okey,
                                                       uint32_t* __restrict__ oval, uint32_t* __restrict__ kcnt,
                                                       uint64_t* __restrict__ ctr, uint32_t* __restrict__ ohist,
                                                       const uint64_t* __restrict__ wsum,
                                                       uint64_t* __restrict__ stamp, uint64_t* __restrict__ ts,
                                                       uint32_t m0_group = 0) {
  constexpr uint32_t CAP = 1u << CAPLOG;
  constexpr uint32_t NB = 1u << DB;  // digit 0 of the order keys (the first ordering pass's digits)
  __shared__ uint64_t s_key[CAP];
  __shared__ uint16_t s_rs[CAP + 1];
  __shared__ uint32_t s_oh[NB];
  __shared__ uint32_t s_w[(NTH / 64)];
  const int t = threadIdx.x;
  const uint32_t b = blockIdx.x;
  ts_enter(ts, TS_HOT_IN);
  sp_stamp(stamp, true, 0);
  if (b == 0 && t == 0) ctr[C_W] = ctr[C_WSORT] = wsum_total(wsum);  // k_sp_exbucket's wedge count
  // after an over-full sub-bucket the call is redone: every bucket reports empty
  const bool abort = (ctr[C_FLAGS] & F_TOOBIG) != 0;
  uint32_t pre[EXB_SUB + 1];  // the bucket's sub-bucket counts, prefix-summed (uniform loads)
  pre[0] = 0;
#pragma unroll
  for (uint32_t q = 0; q < EXB_SUB; ++q) pre[q + 1] = pre[q] + (abort ? 0u : bcnt[b * EXB_SUB + q]);
  const uint32_t m = pre[EXB_SUB];
  if (m == 0 || m > CAP) {  // a bucket beyond the workgroup's sort capacity: the call is redone
    if (t == 0) {
      kcnt[b] = 0;
      if (m > CAP) atomicOr((unsigned long long*)&ctr[C_FLAGS], F_TOOBIG);
    }
    return;
  }
  const uint64_t start = (uint64_t)b * EXB_SUB << CAPLOG;
  for (uint32_t i = t; i < NB; i += NTH) s_oh[i] = 0;
  sp_stamp(stamp, true, 4);
  if (m <= NTH) gr_sort<1, NTH>(rkey, start, m, s_key, t, pre, CAPLOG);
  else if (m <= 2 * NTH) gr_sort<2, NTH>(rkey, start, m, s_key, t, pre, CAPLOG);
  else if (CAP >= 4 * NTH && m <= 4 * NTH)
    gr_sort<(CAP >= 4 * NTH ? 4 : 1), NTH>(rkey, start, m, s_key, t, pre, CAPLOG);
  else if (CAP >= 8 * NTH) gr_sort<(CAP >= 8 * NTH ? 8 : 1), NTH>(rkey, start, m, s_key, t, pre, CAPLOG);
  sp_stamp(stamp, true, 1);
  // run starts (blocked: thread t owns keys [t P, t P + P)) -> run ids -> start positions
  const uint32_t P = (m + NTH - 1) / NTH;
  uint32_t R;
  {
    uint32_t ns = 0;
    for (uint32_t r = 0; r < P; ++r) {
      const uint32_t q = (uint32_t)t * P + r;
      ns += (q < m && (q == 0 || s_key[q - 1] != s_key[q])) ? 1u : 0u;
    }
    uint32_t id = gr_scan<NTH>(ns, s_w, &R);
    for (uint32_t r = 0; r < P; ++r) {
      const uint32_t q = (uint32_t)t * P + r;
      if (q < m && (q == 0 || s_key[q - 1] != s_key[q])) s_rs[id++] = (uint16_t)q;
    }
    if (t == 0) s_rs[R] = (uint16_t)m;
    __syncthreads();
  }
  sp_stamp(stamp, true, 2);
  // score the runs, NTH per round, compacting in run order
  const uint64_t wmask = (1ull << wbits) - 1;
  uint32_t K = 0, nnan = 0;
  for (uint32_t q0 = 0; q0 < R; q0 += NTH) {
    const uint32_t q = q0 + t;
    bool keep = false;
    uint32_t ru = 0, rw = 0;
    float sc = 0.0f;
    if (q < R) {
      const uint32_t p0 = s_rs[q], c = (uint32_t)s_rs[q + 1] - p0;
      const uint64_t key = s_key[p0];
      ru = (uint32_t)(ua + (key >> wbits));
      rw = (uint32_t)(key & wmask);
      const bool ex = first_order(g, ru, rw);
      sc = score_basic(metric, ex ? 0u : c, g.deg[ru], g.deg[rw]);
      keep = !(sc <= min_score) && !f2_drop(g, ru, rw);  // NaN passes
    }
    if (q0 == 0 && stamp) {  // diagnostics: the scoring loads have arrived
      if (keep && sc == -12345.0f) s_w[0] = 1u;
      sp_stamp(stamp, true, 5);
    }
    uint32_t kept;
    const uint32_t pos = K + gr_scan<NTH>(keep ? 1u : 0u, s_w, &kept);
    if (q0 == 0) sp_stamp(stamp, true, 6);
    if (keep) {
      const uint32_t o = (b << CAPLOG) + pos;  // the bucket's candidate slots
      cu[o] = ru;
      cw[o] = rw;
      cs[o] = sc;
      const uint32_t k = ~score_key(sc);
      okey[o] = k;
      oval[o] = o;
      atomicAdd(&s_oh[k & (NB - 1)], 1u);
      nnan += sc != sc;
    }
    K += kept;
  }
  sp_stamp(stamp, true, 7);
  if (t == 0) kcnt[b] = K;
  if (nnan) atomicAdd((unsigned long long*)&ctr[C_NAN], (unsigned long long)nnan);
  __syncthreads();
  // digit 0 into the histogram copies, or (m0_group > 0: counted passes) into
  // row b / m0_group (the bucket's group) of the count matrix m0
  uint32_t* hcp = m0_group ? ohist + (b / m0_group) * NB : hist_copy_db<DB>(ohist);
  for (uint32_t i = t; i < NB; i += NTH) {
    const uint32_t hc = s_oh[i];
    if (hc) atomicAdd(&hcp[i], hc);
  }
  sp_stamp(stamp, true, 3);
}

// ---------------------------------------------------------------- balanced run scoring
// Over the bucket-sorted records, one workgroup per tile of RU_TILE records,
// wave w on records [base + 64 RU_IPT w, +64 RU_IPT): those that start a run
// (rlen > 0) are scored -- first-order exclusion (predict.hxx:306-307), the
// metric, the minScore filter (predict.hxx:311).  No hand-off between
// workgroups: tile t writes its candidates, in record ((u, w)) order, to the
// slots [t RU_TILE, t RU_TILE + seg_cnt[t]) of the candidate columns (a
// "gapped" layout), and the first ordering pass (k_sp_pass<.., GAPPED>) reads
// each tile as one wave segment.  Digit 0 of the order keys is counted.
//
// Exclusion: with the membership table (kernels.hpp et_has) every run costs
// the same two dependent round trips (its key, then table line and degrees);
// without it, the edge filter and a lockstep 4-way search of the shorter of
// N(u) and I(w).
template <bool CUSTOM>
__global__ __launch_bounds__(NT) void k_sp_runs(GraphView g, int metric, float min_score, uint64_t ua, int wbits,
                                                const uint64_t* __restrict__ skey, const uint32_t* __restrict__ rlen,
                                                const uint32_t* __restrict__ vsorted, uint32_t* __restrict__ cu,
                                                uint32_t* __restrict__ cw, float* __restrict__ cs,
                                                uint32_t* __restrict__ okey, uint32_t* __restrict__ oval,
                                                uint32_t* __restrict__ seg_cnt, uint64_t* __restrict__ ctr,
                                                uint32_t* __restrict__ ohist, uint64_t* __restrict__ stamp,
                                                uint64_t* __restrict__ ts) {
  __shared__ uint32_t s_oh[RS_BINS];
  const int t = threadIdx.x, lane = lane_id(), wv = wave_id();
  const uint64_t n = ctr[C_WSORT];
  const uint64_t tile = blockIdx.x;
  if (tile * RU_TILE >= n) return;
  if (ctr[C_FLAGS] & F_TOOBIG) return;  // stale run lengths: the call is redone (the next pass orders nothing)
  ts_enter(ts, TS_HOT_IN);
  s_oh[t] = 0;
  __syncthreads();
  sp_stamp(stamp, true, 0);
  const uint64_t wmask = (1ull << wbits) - 1;
  const uint64_t b0 = tile * RU_TILE + (uint64_t)wv * RU_SEG + lane;
  uint32_t ru[RU_IPT], rw[RU_IPT], rc[RU_IPT], du[RU_IPT], dw[RU_IPT];
  bool has[RU_IPT], ex[RU_IPT];
  float racc[RU_IPT];
#pragma unroll
  for (int j = 0; j < RU_IPT; ++j) {
    const uint64_t i = b0 + (uint64_t)j * 64;
    const bool in = i < n;
    rc[j] = in ? rlen[i] : 0u;
    const uint64_t k = in ? skey[i] : 0ull;
    has[j] = rc[j] != 0;
    ru[j] = (uint32_t)(ua + (k >> wbits));
    rw[j] = (uint32_t)(k & wmask);
  }
#pragma unroll
  for (int j = 0; j < RU_IPT; ++j) {
    const uint64_t i = b0 + (uint64_t)j * 64;
    float acc = 0.0f;
    if (CUSTOM && has[j])  // the reference's order: ascending v
      for (uint32_t q = 0; q < rc[j]; ++q) acc = (float)((double)acc + g.ctab[g.deg[vsorted[i + q]]]);
    racc[j] = acc;
    du[j] = has[j] ? g.deg[ru[j]] : 0u;
    dw[j] = (has[j] && !CUSTOM) ? g.deg[rw[j]] : 0u;
  }
  if (g.etab) {
#pragma unroll
    for (int j = 0; j < RU_IPT; ++j) ex[j] = has[j] && et_has(g.etab, g.etbits, ru[j], rw[j]);
  } else {
    // w in N(u) <=> u in I(w): search the shorter list, lockstep, 4-way
    const bool sym = g.toff == g.off;
    uint32_t lo[RU_IPT], hi[RU_IPT], tg[RU_IPT], ln[RU_IPT];
    const uint32_t* rl[RU_IPT];
#pragma unroll
    for (int j = 0; j < RU_IPT; ++j) {
      rl[j] = g.keys;
      tg[j] = 0;
      ln[j] = 0;
      if (has[j]) {
        const uint64_t ou = g.off[ru[j]];
        const uint64_t tw = g.toff[rw[j]], tw1 = g.toff[rw[j] + 1];
        const uint32_t iw = sym ? dw[j] : (uint32_t)(tw1 - tw);
        const bool via_w = iw < du[j];
        rl[j] = via_w ? g.tkeys + tw : g.keys + ou;
        tg[j] = via_w ? ru[j] : rw[j];
        ln[j] = via_w ? iw : du[j];
        if (g.efbits) {  // not in the edge filter: w is not in N(u), no search
          const uint64_t h = edge_slot(ru[j], rw[j], g.efbits);
          if (!((g.efilt[h >> 5] >> (h & 31)) & 1u)) ln[j] = 0;
        }
      }
      lo[j] = 0;
      hi[j] = ln[j];
    }
    bool more = true;
    while (more) {  // the lower bound lies in [lo, hi]; 3 pivots per round trip
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
    for (int j = 0; j < RU_IPT; ++j) ex[j] = lo[j] < ln[j] && rl[j][lo[j]] == tg[j];
  }
  sp_stamp(stamp, true, 1);
  // wave-local compaction in record order
  uint32_t pos = 0, nnan = 0;
  const uint64_t lt = lane_mask_lt();
  uint32_t sbase = (uint32_t)(tile * RU_TILE + (uint64_t)wv * RU_SEG);
  float sc[RU_IPT];
  bool keep[RU_IPT];
  uint32_t rank[RU_IPT];
#pragma unroll
  for (int j = 0; j < RU_IPT; ++j) {
    sc[j] = 0.0f;
    keep[j] = false;
    if (has[j]) {
      if (CUSTOM) sc[j] = ex[j] ? 0.0f : racc[j];
      else sc[j] = score_basic(metric, ex[j] ? 0u : rc[j], du[j], dw[j]);
      keep[j] = !(sc[j] <= min_score) && !f2_drop(g, ru[j], rw[j]);  // NaN passes
    }
    const uint64_t m = __ballot(keep[j]);
    rank[j] = pos + (uint32_t)__popcll(m & lt);
    pos += (uint32_t)__popcll(m);
  }
  // candidates of wave wv go to its own segment: slots [sbase, sbase + pos)
#pragma unroll
  for (int j = 0; j < RU_IPT; ++j) {
    if (keep[j]) {
      const uint32_t o = sbase + rank[j];
      cu[o] = ru[j];
      cw[o] = rw[j];
      cs[o] = sc[j];
      const uint32_t k = ~score_key(sc[j]);
      okey[o] = k;
      oval[o] = o;
      atomicAdd(&s_oh[k & 0xffu], 1u);
      nnan += sc[j] != sc[j];
    }
  }
  if (lane == 0) seg_cnt[tile * NWAVE + wv] = pos;
  if (nnan) atomicAdd((unsigned long long*)&ctr[C_NAN], (unsigned long long)nnan);
  __syncthreads();
  sp_stamp(stamp, true, 2);
  const uint32_t hc = s_oh[t];
  if (hc) atomicAdd(&hist_copy(ohist)[t], hc);
}

// ---------------------------------------------------------------- generic single-pass scan
// F: count(i) -> u32 (evaluated once, striped), emit(i, off, c).  Ticketed
// tiles (see k_sp_pass); the grand total goes to *total.
template <class F, int IPT>
__global__ __launch_bounds__(NT) void k_sp_scan(F f, const uint64_t* __restrict__ d_n, uint64_t* __restrict__ desc,
                                                uint32_t* __restrict__ tick, uint32_t* __restrict__ err,
                                                uint64_t* __restrict__ total) {
  constexpr int TILE = NT * IPT;
  __shared__ uint32_t s_cnt[TILE];
  __shared__ uint64_t s_red[NWAVE + 1];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_tk[2];
  const uint64_t n = *d_n;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  if (blockIdx.x >= ntiles) return;  // only as many claimants as tiles
  tk_draw(tick, &s_tk[0]);
  __syncthreads();
  for (int par = 0;; par ^= 1) {
    const uint64_t tile = s_tk[par];
    if (tile >= ntiles) break;
    const uint64_t base = tile * TILE;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      const uint64_t j = base + (uint64_t)i * NT + threadIdx.x;
      s_cnt[i * NT + threadIdx.x] = j < n ? f.count(j, n) : 0u;
    }
    __syncthreads();
    tk_draw(tick, &s_tk[par ^ 1]);
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
    const bool excl = first_order(g, u, w);
    float sc;
    if (CUSTOM) sc = excl ? 0.0f : acc;
    else sc = score_basic(metric, excl ? 0u : c, g.deg[u], g.deg[w]);
    stash[i] = sc;
    return (!(sc <= min_score) && !f2_drop(g, u, w)) ? 1u : 0u;  // NaN passes
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
                                                  uint64_t* __restrict__ ctr, uint64_t* __restrict__ hctr,
                                                  const uint64_t* __restrict__ ts,
                                                  uint32_t* __restrict__ clean_desc = nullptr, uint32_t clean_nb = 0,
                                                  uint64_t* __restrict__ sticky = nullptr) {
  const uint64_t m = std::min<uint64_t>(ctr[C_C], k);
  if (clean_desc) {  // the last ordering pass's descriptor rows (clean_nb words each) back to zero (see k_sp_pass)
    const uint64_t words = (ctr[C_C] + OS2_TILE - 1) / OS2_TILE * clean_nb;
    for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < words; i += (uint64_t)gridDim.x * NT)
      clean_desc[i] = 0u;
  }
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) ctr[C_OUT_N] = m;
    if (sticky && threadIdx.x == C_FLAGS) *sticky |= ctr[C_FLAGS];  // see GatherOut::sticky
    if (hctr && threadIdx.x < NCTR) hctr[threadIdx.x] = threadIdx.x == C_OUT_N ? m : ctr[threadIdx.x];
    if (hctr && ts && threadIdx.x >= NCTR && threadIdx.x < NCTR + TS_END) hctr[threadIdx.x] = ts[threadIdx.x - NCTR];
    if (hctr) __threadfence_system();
  }
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < m; i += (uint64_t)gridDim.x * NT) {
    const uint32_t x = idx[i];
    out[i] = EdgeOut{cu[x], cw[x], cs[x]};
  }
  // the call's end (the last-dispatched workgroup's exit, approximately the
  // last one; finding the last one would take one same-address atomic per
  // workgroup, ~0.1 us each, serialised), straight into the host copy
  if (hctr && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    hctr[NCTR + TS_END] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace nlp
