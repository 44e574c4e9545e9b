// Phase timestamps of embed_grad_mfma_kernel<256> (block 0 and the last-started block, thread 0)
// at V=22000, d=256, R=512 (dev tool).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/eg_probe.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ unsigned long long g_probe[512][16];
#define EG_PROBE(k)                                                       \
  do {                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 512) g_probe[blockIdx.x][(k)] = wall_clock64(); \
  } while (0)
#include "embed.hip"

int main() {
  const int V = 22000, d = 256, R = 512, RP = 512;
  void *gT, *xt, *grad, *bg;
  (void)hipMalloc(&gT, (size_t)d * RP * 2);
  (void)hipMalloc(&xt, (size_t)V * (R / 32) * 4);
  (void)hipMalloc(&grad, (size_t)V * d * 4);
  (void)hipMalloc(&bg, d * 4);
  (void)hipMemset(gT, 0, (size_t)d * RP * 2);
  std::vector<uint32_t> bits((size_t)V * (R / 32));
  uint32_t x = 12345;
  for (auto &b : bits) {
    uint32_t w = 0;
    for (int i = 0; i < 32; ++i) { x = x * 1664525u + 1013904223u; if ((x >> 8) % 50 == 0) w |= 1u << i; }
    b = w;
  }
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipMemcpy(xt, bits.data(), bits.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    int rc = cc_embed_grad_mfma(gT, V, d, R, RP, (uint32_t *)xt, (float *)grad, (float *)bg, nullptr);
    (void)hipEventRecord(b);
    (void)hipDeviceSynchronize();
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    static unsigned long long h[512][16];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_probe), sizeof(h));
    unsigned long long t0 = ~0ull, tend = 0;
    for (int i = 0; i < 344; ++i) { t0 = h[i][0] < t0 ? h[i][0] : t0; tend = h[i][15] > tend ? h[i][15] : tend; }
    printf("rep %d rc %d: %.1f us (event), first start -> last end %lld ns\n", rep, rc, ms * 1000, (long long)(tend - t0) * 10);
    for (int i : {0, 1, 100, 255, 256, 300, 343}) {
      printf("  blk %3d start %6lld:", i, (long long)(h[i][0] - t0) * 10);
      for (int k = 1; k < 10; ++k) printf(" %lld", (long long)(h[i][k] - h[i][0]) * 10);
      printf(" end %lld\n", (long long)(h[i][15] - h[i][0]) * 10);
    }
  }
  return 0;
}
