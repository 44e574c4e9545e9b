// Phase timestamps of dec_bce_dw_kernel (block 0, thread 0) at B=512, d=256, V=22000 (dev tool).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/dec_probe.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ unsigned long long g_probe[16];
#define DEC_PROBE(k)                                                              \
  do {                                                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_probe[(k)] = wall_clock64();      \
  } while (0)
#include "decout.hip"

int main() {
  const int B = 512, d = 256, V = 22000, VW = (V + 31) / 32;
  void *D3, *D3t, *D3p, *D3tp, *WoT, *bo, *yb, *dZ, *gW, *gb, *part, *loss, *tick;
  (void)hipMalloc(&D3, B * d * 2);
  (void)hipMalloc(&D3t, B * d * 2);
  (void)hipMalloc(&D3p, B * d * 2);
  (void)hipMalloc(&D3tp, B * d * 2);
  (void)hipMalloc(&WoT, (size_t)V * d * 2);
  (void)hipMalloc(&bo, V * 4);
  (void)hipMalloc(&yb, (size_t)B * VW * 4);
  (void)hipMalloc(&dZ, (size_t)B * V * 2);
  (void)hipMalloc(&gW, (size_t)d * V * 4);
  (void)hipMalloc(&gb, V * 4);
  (void)hipMalloc(&part, 4096 * 8);
  (void)hipMalloc(&loss, 8);
  (void)hipMalloc(&tick, 8);
  for (void *q : {D3, D3t, D3p, D3tp}) (void)hipMemset(q, 0, B * d * 2);
  (void)hipMemset(WoT, 0, (size_t)V * d * 2);
  (void)hipMemset(bo, 0, V * 4);
  (void)hipMemset(yb, 0, (size_t)B * VW * 4);
  (void)hipMemset(tick, 0, 8);
  for (int pk = 0; pk < 2; ++pk) {
    for (int rep = 0; rep < 3; ++rep) {
      int rc = cc_dec_bce_dw(D3, D3t, B, pk ? D3p : nullptr, pk ? D3tp : nullptr, WoT, (const float *)bo, B, d, V,
                             (const uint32_t *)yb, dZ, (float *)gW, (float *)gb, (double *)part, (double *)loss,
                             1.0 / (B * V), (uint32_t *)tick, nullptr);
      (void)hipDeviceSynchronize();
      unsigned long long h[16];
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_probe), sizeof(h));
      printf("packed %d rep %d rc %d:", pk, rep, rc);
      for (int k = 1; k < 9; ++k) printf(" %lld", (long long)(h[k] - h[0]) * 10);
      printf("  (ns: resident, p0 mfma, p0 epi, p1 mfma, p1 epi, sync, ph2 mfma, ph2 stores)\n");
    }
  }
  return 0;
}
