// alloc_probe.hip -- where does hipMalloc time go on the MI355X box?  Times
// hipMalloc / hipFree of large blocks: fresh, after a free of the same size,
// split into smaller blocks, and the first kernel touch (diagnostic for the
// graph build's allocation phase, nlp_graph_build_phases).
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
static void* timed_alloc(size_t bytes, const char* what) {
  void* p = nullptr;
  const double t0 = now_ms();
  hipError_t e = hipMalloc(&p, bytes);
  const double t1 = now_ms();
  printf("%-40s %7.2f GB hipMalloc %8.1f ms (%s)\n", what, bytes / 1e9, t1 - t0, hipGetErrorString(e));
  fflush(stdout);
  return e == hipSuccess ? p : nullptr;
}
static void timed_touch(void* p, size_t bytes, const char* what) {
  const double t0 = now_ms();
  hipLaunchKernelGGL(touch, dim3(8192), dim3(256), 0, 0, (unsigned long long*)p, bytes / 8);
  (void)hipDeviceSynchronize();
  printf("%-40s touch %8.1f ms\n", what, now_ms() - t0);
  fflush(stdout);
}
int main() {
  (void)hipFree(0);
  size_t fr, tot;
  (void)hipMemGetInfo(&fr, &tot);
  printf("free %.1f GB of %.1f GB\n", fr / 1e9, tot / 1e9);
  const size_t GB = 1ull << 30;
  void* a = timed_alloc(1 * GB, "fresh 1 GB");
  void* b = timed_alloc(4 * GB, "fresh 4 GB");
  void* c = timed_alloc(16 * GB, "fresh 16 GB");
  void* d = timed_alloc(34 * GB, "fresh 34 GB");
  timed_touch(d, 34 * GB, "fresh 34 GB");
  timed_touch(d, 34 * GB, "again 34 GB");
  double t0 = now_ms();
  (void)hipFree(d);
  printf("hipFree 34 GB %.1f ms\n", now_ms() - t0);
  d = timed_alloc(34 * GB, "34 GB after freeing 34 GB");
  timed_touch(d, 34 * GB, "reused 34 GB");
  std::vector<void*> parts;
  for (int i = 0; i < 8; ++i) parts.push_back(timed_alloc(4 * GB, "fresh 4 GB part"));
  for (void* p : parts) (void)hipFree(p);
  t0 = now_ms();
  (void)hipFree(c);
  printf("hipFree 16 GB %.1f ms\n", now_ms() - t0);
  void* e = timed_alloc(16 * GB, "16 GB after freeing 16 GB");
  void* f = timed_alloc(64 * GB, "fresh 64 GB");
  (void)hipMemGetInfo(&fr, &tot);
  printf("free %.1f GB\n", fr / 1e9);
  for (void* p : {a, b, d, e, f}) (void)hipFree(p);
  // the graph build's situation: most of HBM in use (touched), then a large block
  std::vector<void*> used;
  for (int i = 0; i < 40; ++i) {
    void* p = timed_alloc(4 * GB, "fill 4 GB");
    if (!p) break;
    timed_touch(p, 4 * GB, "fill 4 GB");
    used.push_back(p);
  }
  (void)hipMemGetInfo(&fr, &tot);
  printf("free %.1f GB\n", fr / 1e9);
  void* g = timed_alloc(34 * GB, "34 GB with 160 GB in use");
  if (g) timed_touch(g, 34 * GB, "34 GB with 160 GB in use");
  void* h = timed_alloc(34 * GB, "another 34 GB");
  if (h) timed_touch(h, 34 * GB, "another 34 GB");
  for (void* p : used) (void)hipFree(p);
  if (g) (void)hipFree(g);
  if (h) (void)hipFree(h);
  return 0;
}
