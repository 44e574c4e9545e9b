// Per-layer timestamps of tower_fwd_fast_kernel (block 0, wave 0, lane 0) at d=256, R=32 (dev tool).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/tower_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ unsigned long long g_probe[32];
#define TOWER_PROBE(k)                                                            \
  do {                                                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_probe[(k)] = wall_clock64();      \
  } while (0)
#include "tower.hip"

int main() {
  const int d = 256, R = 32;
  const int Ks[6] = {d, 256, 128, 64, 128, 256}, Ns[6] = {256, 128, 64, 128, 256, d};
  cc_tower_args t{};
  t.dtype = CC_BF16;
  t.d = d;
  t.B = R;
  t.R = R;
  for (int l = 0; l < 9; ++l) {
    const int i = l < 6 ? l : l - 3;
    void *w, *wt, *b;
    (void)hipMalloc(&w, Ks[i] * Ns[i] * 2);
    (void)hipMalloc(&wt, Ks[i] * Ns[i] * 2);
    (void)hipMalloc(&b, Ns[i] * 4);
    (void)hipMemset(w, 0, Ks[i] * Ns[i] * 2);
    (void)hipMemset(wt, 0, Ks[i] * Ns[i] * 2);
    (void)hipMemset(b, 0, Ns[i] * 4);
    t.w[l] = w;
    t.wt[l] = wt;
    t.b[l] = (const float *)b;
    void *pf, *pb;
    (void)hipMalloc(&pf, Ks[i] * Ns[i] * 2);
    (void)hipMalloc(&pb, Ks[i] * Ns[i] * 2);
    t.wpf[l] = pf;
    t.wpb[l] = pb;
  }
  const int widths[7] = {d, 256, 128, 64, 128, 256, d};
  for (int a = 0; a < 7; ++a) {
    void *x;
    (void)hipMalloc(&x, R * widths[a] * 2);
    (void)hipMemset(x, 0, R * widths[a] * 2);
    t.act[a] = x;
  }
  void *a6t;
  (void)hipMalloc(&a6t, d * R * 2);
  t.act6t = a6t;
  const int freq = 100;  // wall_clock64 MHz on gfx9
  (void)cc_tower_transpose(&t, nullptr);
  for (int rep = 0; rep < 4; ++rep) {
    int rc = cc_tower_fwd(&t, nullptr);
    (void)hipDeviceSynchronize();
    unsigned long long h[32];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_probe), sizeof(h));
    printf("rep %d rc %d:", rep, rc);
    for (int k = 1; k < 20; ++k) printf(" %lld", (long long)(h[k] - h[0]) * 1000 / freq);
    printf("  (ns since start; 1, then per layer: mfma-issued, epilogue, barrier)\n");
  }
  return 0;
}
