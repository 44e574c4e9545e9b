// Phase timestamps of embed_grad_cs_kernel (thread 0 of every block) at V=22000, d=256, R=512
// (dev tool): start skew, staging (all global reads + barrier), per-tile compute + stores, end.
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/eg_cs_probe.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/gpubin/eg_cs_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__device__ unsigned long long g_probe[2048][16];
#define EG_PROBE(k)                                                                         \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 2048) g_probe[blockIdx.x][(k)] = wall_clock64(); \
  } while (0)
#include "embed.hip"

int main() {
  const int V = 22000, d = 256, R = 512, RP = 512;
  void *gP, *xt, *grad, *bg, *tk;
  (void)hipMalloc(&gP, (size_t)d * RP * 2);
  (void)hipMalloc(&xt, (size_t)V * (R / 32) * 4);
  (void)hipMalloc(&grad, (size_t)V * d * 4);
  (void)hipMalloc(&bg, d * 4);
  (void)hipMalloc(&tk, 4096 * 4);
  (void)hipMemset(gP, 0, (size_t)d * RP * 2);
  (void)hipMemset(tk, 0, 4096 * 4);
  std::vector<uint32_t> bits((size_t)V * (R / 32));
  uint32_t x = 12345;
  for (auto &b : bits) {
    uint32_t w = 0;
    for (int i = 0; i < 32; ++i) { x = x * 1664525u + 1013904223u; if ((x >> 8) % 50 == 0) w |= 1u << i; }
    b = w;
  }
  const int nblk = cc_embed_grad_cs_tickets(V, d, R) * (d / 32);
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipMemcpy(xt, bits.data(), bits.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    int rc = cc_embed_grad_cs(gP, 1, V, d, R, RP, (uint32_t *)xt, (float *)grad, (float *)bg, (uint32_t *)tk, nullptr);
    (void)hipEventRecord(b);
    (void)hipDeviceSynchronize();
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    static unsigned long long h[2048][16];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_probe), sizeof(h));
    unsigned long long t0 = ~0ull, tend = 0;
    for (int i = 0; i < nblk; ++i) { t0 = std::min(t0, h[i][0]); tend = std::max(tend, h[i][15]); }
    double st = 0, stg = 0, bar = 0, c1 = 0, mxs = 0, mxe = 0;
    for (int i = 0; i < nblk; ++i) {
      const double s0 = (h[i][0] - t0) * 10.0;
      st += s0; mxs = std::max(mxs, s0);
      stg += (h[i][1] - h[i][0]) * 10.0; bar += (h[i][2] - h[i][1]) * 10.0;
      c1 += (h[i][15] - h[i][2]) * 10.0;
      mxe = std::max(mxe, (h[i][15] - t0) * 10.0);
    }
    printf("rep %d rc %d: %.1f us (event), %d blocks, first start -> last end %.0f ns; mean ns: start %.0f (max %.0f) "
           "staging %.0f barrier %.0f tiles+ticket %.0f\n",
           rep, rc, ms * 1000, nblk, mxe, st / nblk, mxs, stg / nblk, bar / nblk, c1 / nblk);
  }
  return 0;
}
