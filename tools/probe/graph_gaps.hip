// Probe: device-side gap between two dependent kernels for several graph shapes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <time.h>
__global__ void k_mark(unsigned long long* t, int slot, int spin) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[slot * 2] = __builtin_amdgcn_s_memrealtime();
  long c0 = clock64();
  while (clock64() - c0 < spin) {}
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) t[slot * 2 + 1] = __builtin_amdgcn_s_memrealtime();
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
  hipStream_t s, c;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  unsigned long long* t;
  CK(hipMalloc(&t, 64 * 8));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
  CK(hipEventCreate(&e2));
  auto gap = [&](const char* name) {
    std::vector<unsigned long long> h(8);
    hipMemcpy(h.data(), t, 64, hipMemcpyDeviceToHost);
    printf("%-40s k1->k2 gap %.2f us, k2->k3 gap %.2f us\n", name, (h[2] - h[1]) * 0.01, (h[4] - h[3]) * 0.01);
  };
  // A: direct launches
  for (int i = 0; i < 3; ++i) {
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 0, 20000);
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 1, 20000);
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 2, 20000);
    CK(hipStreamSynchronize(s));
  }
  gap("direct");
  for (int i = 0; i < 3; ++i) {
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 0, 20000);
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 1, 20000);
    CK(hipEventRecord(e1, s));
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 2, 20000);
    CK(hipStreamSynchronize(s));
  }
  gap("direct + events (no fence)");
  // B: one captured graph, no events
  hipGraph_t g; hipGraphExec_t x;
  CK(hipStreamBeginCapture(c, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, c, t, 0, 20000);
  hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, c, t, 1, 20000);
  hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, c, t, 2, 20000);
  CK(hipStreamEndCapture(c, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) { CK(hipGraphLaunch(x, s)); CK(hipStreamSynchronize(s)); }
  gap("graph, 3 kernels");
  // C: three single-kernel graphs composed as child nodes with event nodes
  hipGraph_t gk[3];
  for (int k = 0; k < 3; ++k) {
    CK(hipStreamBeginCapture(c, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, c, t, k, 20000);
    CK(hipStreamEndCapture(c, &gk[k]));
  }
  hipGraph_t top; CK(hipGraphCreate(&top, 0));
  hipGraphNode_t prev = nullptr, n;
  CK(hipGraphAddChildGraphNode(&n, top, nullptr, 0, gk[0])); prev = n;
  CK(hipGraphAddEventRecordNode(&n, top, &prev, 1, e0)); prev = n;
  CK(hipGraphAddChildGraphNode(&n, top, &prev, 1, gk[1])); prev = n;
  CK(hipGraphAddEventRecordNode(&n, top, &prev, 1, e1)); prev = n;
  CK(hipGraphAddChildGraphNode(&n, top, &prev, 1, gk[2])); prev = n;
  hipGraphExec_t xc; CK(hipGraphInstantiate(&xc, top, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) { CK(hipGraphLaunch(xc, s)); CK(hipStreamSynchronize(s)); }
  gap("composed children + event nodes");
  // D: composed children, no events
  hipGraph_t top2; CK(hipGraphCreate(&top2, 0));
  prev = nullptr;
  for (int k = 0; k < 3; ++k) { CK(hipGraphAddChildGraphNode(&n, top2, prev ? &prev : nullptr, prev ? 1 : 0, gk[k])); prev = n; }
  hipGraphExec_t xd; CK(hipGraphInstantiate(&xd, top2, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) { CK(hipGraphLaunch(xd, s)); CK(hipStreamSynchronize(s)); }
  gap("composed children, no events");
  // E: graph with kernel nodes + event nodes directly (flattened)
  hipGraph_t top3; CK(hipGraphCreate(&top3, 0));
  prev = nullptr;
  for (int k = 0; k < 3; ++k) {
    size_t nn = 0; CK(hipGraphGetNodes(gk[k], nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn); CK(hipGraphGetNodes(gk[k], nodes.data(), &nn));
    hipKernelNodeParams kp; CK(hipGraphKernelNodeGetParams(nodes[0], &kp));
    CK(hipGraphAddKernelNode(&n, top3, prev ? &prev : nullptr, prev ? 1 : 0, &kp)); prev = n;
    if (k < 2) { CK(hipGraphAddEventRecordNode(&n, top3, &prev, 1, k ? e1 : e0)); prev = n; }
  }
  hipGraphExec_t xe; CK(hipGraphInstantiate(&xe, top3, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) { CK(hipGraphLaunch(xe, s)); CK(hipStreamSynchronize(s)); }
  gap("flat kernel nodes + event nodes");
  float ms = -1; CK(hipEventElapsedTime(&ms, e0, e1)); printf("  e0->e1 %.2f us\n", ms * 1000);
  // host round trip of a trivial graph launch + sync
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto t0 = clock();
  for (int i = 0; i < 200; ++i) { CK(hipGraphLaunch(x, s)); CK(hipStreamSynchronize(s)); }
  printf("graph launch+sync x200: %.2f us per call (3 kernels of ~8us)\n", (double)(clock() - t0) / CLOCKS_PER_SEC / 200 * 1e6);
  t0 = clock();
  for (int i = 0; i < 200; ++i) { CK(hipGraphLaunch(x, s)); while (hipStreamQuery(s) == hipErrorNotReady) {} }
  printf("graph launch+spin x200: %.2f us per call\n", (double)(clock() - t0) / CLOCKS_PER_SEC / 200 * 1e6);
  t0 = clock();
  for (int i = 0; i < 200; ++i) {
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 0, 20000);
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 1, 20000);
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 2, 20000);
    CK(hipStreamSynchronize(s));
  }
  printf("direct 3 launches+sync x200: %.2f us per call\n", (double)(clock() - t0) / CLOCKS_PER_SEC / 200 * 1e6);
  t0 = clock();
  for (int i = 0; i < 200; ++i) {
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 0, 20000);
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 1, 20000);
    hipLaunchKernelGGL(k_mark, dim3(256), dim3(256), 0, s, t, 2, 20000);
    CK(hipEventRecord(e2, s));
    while (hipEventQuery(e2) == hipErrorNotReady) {}
  }
  printf("direct 3 launches+event spin x200: %.2f us per call\n", (double)(clock() - t0) / CLOCKS_PER_SEC / 200 * 1e6);
  t0 = clock();
  for (int i = 0; i < 200; ++i) { CK(hipGraphLaunch(xe, s)); CK(hipEventRecord(e2, s)); while (hipEventQuery(e2) == hipErrorNotReady) {} }
  printf("flat graph+event spin x200: %.2f us per call\n", (double)(clock() - t0) / CLOCKS_PER_SEC / 200 * 1e6);
  // device time of the 3 kernels alone
  std::vector<unsigned long long> h(8);
  hipMemcpy(h.data(), t, 64, hipMemcpyDeviceToHost);
  printf("device span of 3 kernels: %.2f us\n", (h[5] - h[0]) * 0.01);
  return 0;
}
