// bucket.hip -- micro-benchmark of k_sp_bucket on synthetic records (phase stamps).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/bucket.hip -o tools/ubench/bucket
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include "../../neighborhood-link-prediction-openmp_amd/csrc/sortpath.hpp"
using namespace nlp;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t xr() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }

int main(int argc, char** argv) {
  const int per = argc > 1 ? atoi(argv[1]) : 960;   // records per bucket (mean)
  const int hub = argc > 2 ? atoi(argv[2]) : 0;     // extra records of one hub u in bucket 7
  const uint64_t S = 1ull << 23;
  const int wbits = 23, ubits = 23;
  const int shift = wbits + ubits - 8;
  // graph: every vertex has 4 random neighbours, vertex 12345 has 100000
  std::vector<uint64_t> off(S + 1);
  std::vector<uint32_t> deg(S);
  uint64_t m = 0;
  for (uint64_t v = 0; v < S; ++v) { off[v] = m; deg[v] = v == 12345 ? 100000 : 4; m += deg[v]; }
  off[S] = m;
  std::vector<uint32_t> keys(m);
  for (uint64_t v = 0; v < S; ++v) {
    for (uint64_t j = off[v]; j < off[v + 1]; ++j) keys[j] = (uint32_t)(xr() % S);
    std::sort(keys.begin() + off[v], keys.begin() + off[v + 1]);
  }
  // records: bucket b gets `per` records with u in [b << 15, (b+1) << 15)
  std::vector<uint64_t> rk;
  std::vector<uint32_t> rv;
  std::vector<uint32_t> hist(256, 0);
  for (int b = 0; b < 256; ++b) {
    int cnt = per + (int)(xr() % (per / 4 + 1)) - per / 8 + (b == 7 ? hub : 0);
    for (int i = 0; i < cnt; ++i) {
      uint64_t u = ((uint64_t)b << 15) | (xr() & 0x7fff);
      if (b == 7 && i < hub) u = (7ull << 15) | 100;  // hub-like: one u, many w
      uint64_t w = xr() % S;
      rk.push_back((u << wbits) | w);
      rv.push_back((uint32_t)(xr() % S));
    }
    hist[b] = cnt;
  }
  const uint64_t W = rk.size();
  printf("W=%llu per=%d hub=%d\n", (unsigned long long)W, per, hub);
  uint64_t *d_off, *d_rk, *d_ctr, *d_desc, *d_stamp;
  uint32_t *d_keys, *d_deg, *d_rv, *d_hist, *cu, *cw, *ok, *ov, *oh;
  float* cs;
  CK(hipMalloc(&d_off, (S + 1) * 8)); CK(hipMalloc(&d_keys, m * 4)); CK(hipMalloc(&d_deg, S * 4));
  CK(hipMalloc(&d_rk, W * 8)); CK(hipMalloc(&d_rv, W * 4)); CK(hipMalloc(&d_hist, HCOPIES * HSTRIDE * 4));
  CK(hipMemset(d_hist, 0, HCOPIES * HSTRIDE * 4));
  CK(hipMalloc(&cu, W * 4)); CK(hipMalloc(&cw, W * 4)); CK(hipMalloc(&cs, W * 4)); CK(hipMalloc(&ok, W * 4));
  CK(hipMalloc(&ov, W * 4)); CK(hipMalloc(&oh, HCOPIES * HSTRIDE * 4)); CK(hipMalloc(&d_ctr, 16 * 8));
  CK(hipMalloc(&d_desc, 260 * 8)); CK(hipMalloc(&d_stamp, 256 * 8 * 8));
  CK(hipMemcpy(d_off, off.data(), (S + 1) * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_keys, keys.data(), m * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_deg, deg.data(), S * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rk, rk.data(), W * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rv, rv.data(), W * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_hist, hist.data(), 256 * 4, hipMemcpyHostToDevice));
  GraphView gv{d_off, d_keys, d_deg, d_off, d_keys, nullptr};
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int rep = 0; rep < 12; ++rep) {
    uint64_t h[16] = {};
    h[C_WSORT] = W;
    CK(hipMemcpy(d_ctr, h, 128, hipMemcpyHostToDevice));
    CK(hipMemset(d_desc, 0, 260 * 8));
    CK(hipMemset(oh, 0, HCOPIES * HSTRIDE * 4));
    CK(hipMemset(d_stamp, 0, 256 * 64));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_sp_bucket<false>, dim3(256), dim3(BK_NT), 0, 0, gv, 1, 0.0f, (uint64_t)0, wbits,
                       (const uint64_t*)d_rk, (const uint32_t*)d_rv, (const uint32_t*)d_hist, cu, cw, cs, ok, ov,
                       d_desc, d_ctr, shift, (uint64_t)W, oh, d_stamp);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms * 1000);
  }
  std::sort(ts.begin(), ts.end());
  uint64_t h[16];
  CK(hipMemcpy(h, d_ctr, 128, hipMemcpyDeviceToHost));
  printf("k_sp_bucket: median %.2f us  C=%llu flags=%llx\n", ts[ts.size() / 2], (unsigned long long)h[C_C],
         (unsigned long long)h[C_FLAGS]);
  std::vector<uint64_t> st(256 * 8);
  CK(hipMemcpy(st.data(), d_stamp, st.size() * 8, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull;
  for (int i = 0; i < 256; ++i) t0 = std::min(t0, st[i * 8]);
  const char* nm[7] = {"start", "bounds", "load", "sort", "score", "lookback", "emit"};
  for (int p = 1; p < 7; ++p) {
    double s = 0, mx = 0;
    for (int i = 0; i < 256; ++i) {
      double d = (st[i * 8 + p] - st[i * 8 + p - 1]) * 0.01;
      s += d;
      mx = std::max(mx, d);
    }
    printf("  %-8s mean %6.2f  max %6.2f us\n", nm[p], s / 256, mx);
  }
  // verify: candidates sorted by (u, w) strictly increasing
  std::vector<uint32_t> hu(h[C_C]), hw(h[C_C]);
  CK(hipMemcpy(hu.data(), cu, hu.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hw.data(), cw, hw.size() * 4, hipMemcpyDeviceToHost));
  uint64_t bad = 0;
  for (size_t i = 1; i < hu.size(); ++i)
    if (((uint64_t)hu[i] << 32 | hw[i]) <= ((uint64_t)hu[i - 1] << 32 | hw[i - 1])) ++bad;
  // expected distinct keys
  std::vector<uint64_t> sk = rk;
  std::sort(sk.begin(), sk.end());
  uint64_t distinct = std::unique(sk.begin(), sk.end()) - sk.begin();
  printf("order violations %llu, distinct keys %llu (candidates <= distinct)\n", (unsigned long long)bad,
         (unsigned long long)distinct);
  return 0;
}
