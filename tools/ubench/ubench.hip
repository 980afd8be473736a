// ubench.hip -- micro-benchmarks of the sort-path building blocks on one MI355X.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/ubench.hip -o tools/ubench/ubench
//   ./tools/ubench/ubench            (prints one line per case, times in us)
//
// Each case is timed with HIP events around a single launch (median of 15).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#include "../../neighborhood-link-prediction-openmp_amd/csrc/sortpath.hpp"

using namespace nlp;

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1000) *p = 1;
}

__global__ __launch_bounds__(256) void k_stream_sum(const uint4* __restrict__ a, uint64_t n4, uint32_t* out) {
  uint32_t s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
    uint4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 0xdeadbeef) *out = s;
}

struct Timer {
  hipEvent_t a, b;
  Timer() {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
  template <class F, class P>
  float median(F launch, P prep, int reps = 15) {
    std::vector<float> v;
    for (int r = 0; r < reps; ++r) {
      prep();
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      v.push_back(ms * 1000.f);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  }
};

static uint64_t rng = 88172645463325252ull;
static uint64_t xs() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

// Phase report from per-workgroup s_memrealtime stamps (10 ns ticks).
void report_stamps(const char* tag, uint64_t* d_stamp, unsigned blocks, int nph) {
  std::vector<uint64_t> h((size_t)blocks * 8);
  CK(hipMemcpy(h.data(), d_stamp, h.size() * 8, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull, tend = 0;
  for (unsigned b = 0; b < blocks; ++b) {
    t0 = std::min(t0, h[b * 8]);
    tend = std::max(tend, h[b * 8 + nph - 1]);
  }
  printf("   %s phases (us, mean over %u blocks; start offset, then per phase):", tag, blocks);
  double st = 0;
  for (unsigned b = 0; b < blocks; ++b) st += (h[b * 8] - t0) * 0.01;
  printf(" start+%.2f", st / blocks);
  for (int i = 1; i < nph; ++i) {
    double a = 0, mx = 0;
    for (unsigned b = 0; b < blocks; ++b) {
      double d = (h[b * 8 + i] - h[b * 8 + i - 1]) * 0.01;
      a += d;
      mx = std::max(mx, d);
    }
    printf(" | p%d %.2f (max %.2f)", i, a / blocks, mx);
  }
  printf(" | span %.2f\n", (tend - t0) * 0.01);
}

int occ_of(const void* k) {
  int nb = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, NT, 0));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  return nb * p.multiProcessorCount;
}

template <int IPT, int WIDE>
void launch_pass(unsigned grid, uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint64_t* dn, uint32_t* hist,
                 uint32_t* desc, uint32_t* err, uint64_t* stamp) {
  if (WIDE == 4)
    hipLaunchKernelGGL((k_sp_pass3<uint64_t, IPT, 32>), dim3(grid), dim3(512), 0, 0, (const uint64_t*)k0,
                       (const uint32_t*)v0, k1, v1, (const uint64_t*)dn, 0, (const uint32_t*)hist, desc, err, stamp,
                       (uint32_t*)nullptr);
  else if (WIDE == 2)
    hipLaunchKernelGGL((k_sp_pass2<uint64_t, 512, IPT, 32>), dim3(grid), dim3(512), 0, 0, (const uint64_t*)k0,
                       (const uint32_t*)v0, k1, v1, (const uint64_t*)dn, 0, (const uint32_t*)hist, desc, err, stamp);
  else if (WIDE == 3)
    hipLaunchKernelGGL((k_sp_pass2<uint64_t, 256, IPT, 64>), dim3(grid), dim3(256), 0, 0, (const uint64_t*)k0,
                       (const uint32_t*)v0, k1, v1, (const uint64_t*)dn, 0, (const uint32_t*)hist, desc, err, stamp);
  else if (WIDE == 1)
    hipLaunchKernelGGL((k_sp_passb<uint64_t, IPT>), dim3(grid), dim3(OSB_NT), 0, 0, (const uint64_t*)k0,
                       (const uint32_t*)v0, k1, v1, (const uint64_t*)dn, 0, (const uint32_t*)hist, desc, err, stamp);
  else
    hipLaunchKernelGGL((k_sp_pass<uint64_t, IPT>), dim3(grid), dim3(NT), 0, 0, (const uint64_t*)k0,
                       (const uint32_t*)v0, k1, v1, (const uint64_t*)dn, 0, (const uint32_t*)hist, desc, err, stamp,
                       GatherOut{});
}

template <int IPT, int WIDE>
void bench_pass(Timer& T, uint64_t n, int nbits, bool prefill) {
  constexpr int BT = WIDE == 1 ? OSB_NT : (WIDE == 2 || WIDE == 4) ? 512 : NT;
  auto kern = WIDE == 1   ? (const void*)k_sp_passb<uint64_t, IPT>
              : WIDE == 2 ? (const void*)k_sp_pass2<uint64_t, 512, IPT, 32>
              : WIDE == 3 ? (const void*)k_sp_pass2<uint64_t, 256, IPT, 64>
              : WIDE == 4 ? (const void*)k_sp_pass3<uint64_t, IPT, 32>
                          : (const void*)k_sp_pass<uint64_t, IPT>;
  std::vector<uint64_t> hk(n);
  std::vector<uint32_t> hv(n);
  for (uint64_t i = 0; i < n; ++i) {
    hk[i] = xs() & ((1ull << nbits) - 1);
    hv[i] = (uint32_t)i;
  }
  uint64_t *k0, *k1, *dn, *stamp;
  uint32_t *v0, *v1, *hist, *desc, *err;
  const uint64_t tiles = (n + BT * IPT - 1) / (BT * IPT);
  CK(hipMalloc(&k0, n * 8));
  CK(hipMalloc(&k1, n * 8));
  CK(hipMalloc(&v0, n * 4));
  CK(hipMalloc(&v1, n * 4));
  CK(hipMalloc(&hist, HCOPIES * HSTRIDE * 4));
  CK(hipMalloc(&desc, tiles * 256 * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&dn, 8));
  CK(hipMalloc(&stamp, tiles * 8 * 8));
  CK(hipMemcpy(k0, hk.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dn, &n, 8, hipMemcpyHostToDevice));
  CK(hipMemset(hist, 0, HCOPIES * HSTRIDE * 4));
  CK(hipMemset(err, 0, 4));
  hipLaunchKernelGGL(k_sp_hist<uint64_t>, dim3(128), dim3(NT), 0, 0, (const uint64_t*)k0, (const uint64_t*)dn,
                     n, 0, 1, hist, (uint64_t*)nullptr, (uint64_t*)nullptr);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> pre(tiles * 256, 2u << 30);
  int nb = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, BT, 0));
  const int occ = nb * 256;
  const unsigned grid = (unsigned)std::min<uint64_t>(tiles, occ);
  float us = T.median(
      [&] {
        launch_pass<IPT, WIDE>(grid, k0, v0, k1, v1, dn, hist, desc, err, (uint64_t*)nullptr);
      },
      [&] {
        if (prefill) CK(hipMemcpy(desc, pre.data(), tiles * 256 * 4, hipMemcpyHostToDevice));
        else CK(hipMemset(desc, 0, tiles * 256 * 4));
        CK(hipDeviceSynchronize());
      });
  // check the digit-0 order once (normal mode)
  bool ok = true;
  if (!prefill) {
    std::vector<uint64_t> out(n);
    CK(hipMemcpy(out.data(), k1, n * 8, hipMemcpyDeviceToHost));
    for (uint64_t i = 1; i < n; ++i)
      if ((out[i] & 255) < (out[i - 1] & 255)) { ok = false; break; }
  }
  printf("pass%s<u64,IPT=%2d> n=%9llu tiles=%6llu grid=%5u %s: %8.2f us  %s\n", WIDE == 1 ? "B" : WIDE == 2 ? "2/512" : WIDE == 3 ? "2/256" : WIDE == 4 ? "3/512" : "", IPT,
         (unsigned long long)n,
         (unsigned long long)tiles, grid, prefill ? "lookback-free" : "full         ", us, ok ? "" : "ORDER BAD");
  if (prefill) CK(hipMemcpy(desc, pre.data(), tiles * 256 * 4, hipMemcpyHostToDevice));
  else CK(hipMemset(desc, 0, tiles * 256 * 4));
  CK(hipDeviceSynchronize());
  launch_pass<IPT, WIDE>(grid, k0, v0, k1, v1, dn, hist, desc, err, stamp);
  CK(hipDeviceSynchronize());
  report_stamps("load|rank|lookback|scatter", stamp, grid, 5);
  hipFree(k0); hipFree(k1); hipFree(v0); hipFree(v1); hipFree(hist); hipFree(desc); hipFree(err); hipFree(dn);
  hipFree(stamp);
}

template <int STEPS>
void bench_surv(Timer& T, uint64_t S, double frac) {
  std::vector<uint32_t> hd(S);
  for (uint64_t i = 0; i < S; ++i) hd[i] = (xs() % 1000000) < frac * 1e6 ? 3 : 20;
  uint32_t *deg, *surv;
  uint64_t *desc, *ctr, *stamp;
  const uint64_t tiles = (S + NT * 4 * STEPS - 1) / (NT * 4 * STEPS);
  CK(hipMalloc(&stamp, tiles * 8 * 8));
  CK(hipMalloc(&deg, S * 4));
  CK(hipMalloc(&surv, S * 4));
  CK(hipMalloc(&desc, (tiles + 1) * 8));
  CK(hipMalloc(&ctr, 16 * 8));
  CK(hipMemcpy(deg, hd.data(), S * 4, hipMemcpyHostToDevice));
  const int occ = occ_of((const void*)k_sp_survivors<STEPS>);
  const unsigned grid = (unsigned)std::min<uint64_t>(tiles, occ);
  float us = T.median(
      [&] {
        hipLaunchKernelGGL(k_sp_survivors<STEPS>, dim3(grid), dim3(NT), 0, 0, (const uint32_t*)deg, S, 4u, surv,
                           desc, ctr, (uint64_t*)nullptr);
      },
      [&] {
        CK(hipMemset(desc, 0, (tiles + 1) * 8));
        CK(hipMemset(ctr, 0, 16 * 8));
        CK(hipDeviceSynchronize());
      });
  uint64_t h[16];
  CK(hipMemcpy(h, ctr, 128, hipMemcpyDeviceToHost));
  uint64_t want = 0;
  for (auto d : hd) want += d <= 4;
  printf("survivors<STEPS=%2d> S=%9llu tiles=%6llu grid=%5u: %8.2f us (%.0f GB/s)  nv=%llu %s\n", STEPS,
         (unsigned long long)S, (unsigned long long)tiles, grid, us, S * 4 / us / 1e3, (unsigned long long)h[C_NV],
         h[C_NV] == want ? "" : "COUNT BAD");
  CK(hipMemset(desc, 0, (tiles + 1) * 8));
  CK(hipMemset(ctr, 0, 16 * 8));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_sp_survivors<STEPS>, dim3(grid), dim3(NT), 0, 0, (const uint32_t*)deg, S, 4u, surv, desc, ctr,
                     stamp);
  CK(hipDeviceSynchronize());
  report_stamps("load|lookback|emit", stamp, grid, 4);
  hipFree(deg); hipFree(surv); hipFree(desc); hipFree(ctr); hipFree(stamp);
}

int main() {
  Timer T;
  float e = T.median([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, (int*)nullptr); }, [] {});
  printf("empty kernel (1 block): %.2f us\n", e);
  e = T.median([&] { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, 0, (int*)nullptr); }, [] {});
  printf("empty kernel (1024 blocks): %.2f us\n", e);
  for (uint64_t mb : {19ull, 64ull, 256ull, 1024ull}) {
    uint64_t n = mb << 20;
    uint4* a;
    uint32_t* o;
    CK(hipMalloc(&a, n));
    CK(hipMalloc(&o, 4));
    CK(hipMemset(a, 1, n));
    for (unsigned g : {1024u, 4096u}) {
      float us = T.median([&] { hipLaunchKernelGGL(k_stream_sum, dim3(g), dim3(256), 0, 0, (const uint4*)a, n / 16, o); },
                          [] {});
      printf("stream read %4llu MB grid %5u: %8.2f us  %.0f GB/s\n", (unsigned long long)mb, g, us, n / us / 1e3);
    }
    hipFree(a);
    hipFree(o);
  }
  bench_surv<8>(T, 4847572, 0.02);
  bench_surv<4>(T, 4847572, 0.02);
  for (uint64_t n : {245525ull, 1000000ull, 4000000ull}) {
    bench_pass<16, 0>(T, n, 46, false);
    bench_pass<8, 4>(T, n, 46, false);
    bench_pass<4, 4>(T, n, 46, false);
  }
  return 0;
}
