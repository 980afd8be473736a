// Probe: can a captured hipGraph carry timing events (hipEventRecordExternal)?
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k_spin(int* p, int n) {
  long t0 = clock64();
  while (clock64() - t0 < n) {}
  if (p && threadIdx.x == 9999) *p = 1;
}
#define P(x) do { hipError_t e = (x); printf("%-60s -> %s\n", #x, hipGetErrorString(e)); } while (0)
int main() {
  hipStream_t s, c;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&c, hipStreamNonBlocking);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipGraph_t g = nullptr;
  hipGraphExec_t x = nullptr;
  P(hipStreamBeginCapture(c, hipStreamCaptureModeThreadLocal));
  P(hipEventRecordWithFlags(a, c, hipEventRecordExternal));
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, c, (int*)nullptr, 200000);
  P(hipEventRecordWithFlags(b, c, hipEventRecordExternal));
  P(hipStreamEndCapture(c, &g));
  P(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) {
    P(hipGraphLaunch(x, s));
    P(hipStreamSynchronize(s));
    float ms = -1;
    P(hipEventElapsedTime(&ms, a, b));
    printf("elapsed %.3f ms\n", ms);
  }
  // plain hipEventRecord inside capture
  hipGraph_t g2 = nullptr;
  hipGraphExec_t x2 = nullptr;
  P(hipStreamBeginCapture(c, hipStreamCaptureModeThreadLocal));
  P(hipEventRecord(a, c));
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, c, (int*)nullptr, 200000);
  P(hipEventRecord(b, c));
  P(hipStreamEndCapture(c, &g2));
  P(hipGraphInstantiate(&x2, g2, nullptr, nullptr, 0));
  P(hipGraphLaunch(x2, s));
  P(hipStreamSynchronize(s));
  float ms = -1;
  P(hipEventElapsedTime(&ms, a, b));
  printf("elapsed (plain record in capture) %.3f ms\n", ms);
  // host launch overhead: 200 launches of a 4-kernel graph vs direct
  return 0;
}
