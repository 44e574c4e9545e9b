// Phase timestamps of kl_main_kernel (block 0, thread 0) at 512 rows, d = 256, V = 22000 (dev tool).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/kl_probe.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/kl_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ unsigned long long g_probe[16];
#define KL_PROBE(k)                                                               \
  do {                                                                            \
    if (sl == 0 && threadIdx.x == 0) g_probe[(k)] = wall_clock64();              \
  } while (0)
#include "decreg.hip"

int main() {
  const int rows = 512, B = 512, R = B + rows, d = 256, V = 22000;
  void *D3p, *D3tp, *Wo, *bo, *Mt, *tsum, *ridx, *dZ, *gW, *gb, *part, *loss, *tick, *ws;
  (void)hipMalloc(&D3p, (size_t)R * d * 2);
  (void)hipMalloc(&D3tp, (size_t)R * d * 2);
  (void)hipMalloc(&Wo, (size_t)V * d * 2);
  (void)hipMalloc(&bo, V * 4);
  (void)hipMalloc(&Mt, (size_t)V * V * 4);
  (void)hipMalloc(&tsum, V * 4);
  (void)hipMalloc(&ridx, rows * 4);
  (void)hipMalloc(&dZ, (size_t)rows * V * 2);
  (void)hipMalloc(&gW, (size_t)d * V * 4);
  (void)hipMalloc(&gb, V * 4);
  (void)hipMalloc(&part, 4096 * 8);
  (void)hipMalloc(&loss, 8);
  (void)hipMalloc(&tick, 8);
  (void)hipMalloc(&ws, cc_dec_kl_ws_size(rows, V));
  for (void *q : {D3p, D3tp}) (void)hipMemset(q, 0, (size_t)R * d * 2);
  (void)hipMemset(Wo, 0, (size_t)V * d * 2);
  (void)hipMemset(bo, 0, V * 4);
  (void)hipMemset(Mt, 0, (size_t)V * V * 4);
  (void)hipMemset(tsum, 0, V * 4);
  (void)hipMemset(tick, 0, 8);
  std::vector<int> h(rows);
  for (int i = 0; i < rows; ++i) h[i] = (i * 7919) % V;
  (void)hipMemcpy(ridx, h.data(), rows * 4, hipMemcpyHostToDevice);
  cc_dec_kl_args a{};
  a.d = d; a.V = V; a.rows = rows; a.ldt = R; a.row0 = B;
  a.D3p = D3p; a.D3tp = D3tp; a.Wo = Wo; a.bo = (const float *)bo; a.Mt = (const float *)Mt;
  a.tsum = (const float *)tsum; a.mt_bytes = (int64_t)V * V * 4; a.mt_lo = 0; a.reg_idx = (const int32_t *)ridx;
  a.scale = 1e-4f; a.dZ = dZ; a.gW = (float *)gW; a.gb = (float *)gb; a.loss_partials = (double *)part;
  a.loss_out = (double *)loss; a.loss_scale = 1.0 / rows; a.ticket = (uint32_t *)tick; a.ws = ws;
  for (int rep = 0; rep < 4; ++rep) {
    int rc = cc_dec_softmax_kl_dw(&a, nullptr);
    (void)hipDeviceSynchronize();
    unsigned long long g[16];
    (void)hipMemcpyFromSymbol(g, HIP_SYMBOL(g_probe), sizeof(g));
    printf("rep %d rc %d:", rep, rc);
    for (int k = 1; k < 8; ++k) printf(" %lld", (long long)(g[k] - g[0]) * 10);
    printf("  (ns: staged, p0 logits, p0 epi, p1 logits, p1 epi, pre-ph2, end)\n");
    printf("   stats:");
    for (int k = 9; k < 12; ++k) printf(" %lld", (long long)(g[k] - g[8]) * 10);
    printf("  (ns: Wo slice staged, logits+lane max, row max/sum reductions)\n");
  }
  return 0;
}
