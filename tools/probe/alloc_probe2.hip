// alloc_probe2.hip -- does allocating right after freeing a lot of HBM wait?
// Fill 160 GB (touched), free it, then allocate + touch 4-GB blocks, timing
// each, and poll hipMemGetInfo (diagnostic for the graph build's allocation
// stalls right after torch hands its cache back).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
__global__ void touch(unsigned long long* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = i;
}
int main() {
  (void)hipFree(0);
  const size_t GB = 1ull << 30;
  size_t fr, tot;
  std::vector<void*> used;
  for (int i = 0; i < 40; ++i) {
    void* p = nullptr;
    if (hipMalloc(&p, 4 * GB) != hipSuccess) break;
    hipLaunchKernelGGL(touch, dim3(4096), dim3(256), 0, 0, (unsigned long long*)p, 4 * GB / 8);
    used.push_back(p);
  }
  (void)hipDeviceSynchronize();
  (void)hipMemGetInfo(&fr, &tot);
  printf("filled %zu x 4 GB, free %.1f GB\n", used.size(), fr / 1e9);
  const double t0 = now_ms();
  for (void* p : used) (void)hipFree(p);
  printf("freed in %.1f ms\n", now_ms() - t0);
  (void)hipMemGetInfo(&fr, &tot);
  printf("free right after: %.1f GB\n", fr / 1e9);
  std::vector<void*> again;
  for (int i = 0; i < 40; ++i) {
    void* p = nullptr;
    const double a = now_ms();
    const hipError_t e = hipMalloc(&p, 4 * GB);
    const double b = now_ms();
    if (e != hipSuccess) { printf("alloc %d failed\n", i); break; }
    hipLaunchKernelGGL(touch, dim3(4096), dim3(256), 0, 0, (unsigned long long*)p, 4 * GB / 8);
    (void)hipDeviceSynchronize();
    const double c = now_ms();
    (void)hipMemGetInfo(&fr, &tot);
    printf("t=%7.1f ms alloc #%2d %8.1f ms touch %7.1f ms free %.1f GB\n", c - t0, i, b - a, c - b, fr / 1e9);
    fflush(stdout);
    again.push_back(p);
  }
  for (void* p : again) (void)hipFree(p);
  for (int i = 0; i < 20; ++i) {
    (void)hipMemGetInfo(&fr, &tot);
    printf("t=%7.1f ms free %.1f GB\n", now_ms() - t0, fr / 1e9);
    const double w = now_ms();
    while (now_ms() - w < 250) {}
  }
  return 0;
}
