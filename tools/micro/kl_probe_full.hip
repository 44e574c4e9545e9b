// Phase totals of kl_main_kernel (block 0, thread 0) over all row tiles, full-mode shape by default
// (rows = |V| identity rows, d = 256, V = 22000): time between consecutive KL_PROBE points summed
// into the later point's bucket (dev tool).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/kl_probe_full.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/gpubin/kl_probe_full
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ unsigned long long g_acc[16], g_last, g_cnt[16];
#define KL_PROBE(k)                                                   \
  do {                                                                \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                        \
      const unsigned long long now = wall_clock64();                  \
      if ((k) != 0 && (k) != 8) { g_acc[(k)] += now - g_last; g_cnt[(k)] += 1; } \
      g_last = now;                                                   \
    }                                                                 \
  } while (0)
#include "decreg.hip"

int main(int argc, char **argv) {
  const int V = 22000, d = 256;
  const int rows = argc > 1 ? atoi(argv[1]) : 22016, B = 512, R = B + rows;
  void *D3p, *D3tp, *Wo, *bo, *Mt, *tsum, *ridx, *dZ, *gW, *gb, *part, *loss, *tick, *ws;
  (void)hipMalloc(&D3p, (size_t)R * d * 2);
  (void)hipMalloc(&D3tp, (size_t)R * d * 2);
  (void)hipMalloc(&Wo, (size_t)V * d * 2);
  (void)hipMalloc(&bo, V * 4);
  (void)hipMalloc(&Mt, (size_t)V * V * 4);
  (void)hipMalloc(&tsum, V * 8);
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
  (void)hipMemset(tsum, 0, V * 8);
  (void)hipMemset(tick, 0, 8);
  std::vector<int> h(rows);
  for (int i = 0; i < rows; ++i) h[i] = i < V ? i : -1;
  (void)hipMemcpy(ridx, h.data(), rows * 4, hipMemcpyHostToDevice);
  cc_dec_kl_args a{};
  a.d = d; a.V = V; a.rows = rows; a.ldt = R; a.row0 = B;
  a.D3p = D3p; a.D3tp = D3tp; a.Wo = Wo; a.bo = (const float *)bo; a.Mt = (const float *)Mt;
  a.tsum = (const float *)tsum; a.mt_bytes = (int64_t)V * V * 4; a.mt_lo = 0; a.reg_idx = (const int32_t *)ridx;
  a.scale = 1e-4f; a.dZ = dZ; a.gW = (float *)gW; a.gb = (float *)gb; a.loss_partials = (double *)part;
  a.loss_out = (double *)loss; a.loss_scale = 1.0 / rows; a.ticket = (uint32_t *)tick; a.ws = ws;
  a.flags = argc > 2 ? atoi(argv[2]) : 0;   // cc_dec_kl_args.flags (A/B of the main pass's paths)
  const char *names[8] = {"", "tile stats staged", "p0 logits", "p0 epilogue", "p1 logits", "p1 epilogue", "phase-2 wait", "phase 2 (+last)"};
  for (int rep = 0; rep < 3; ++rep) {
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_acc), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_cnt), z, sizeof(z));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    int rc = cc_dec_softmax_kl_dw(&a, nullptr);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long g[16], c[16];
    (void)hipMemcpyFromSymbol(g, HIP_SYMBOL(g_acc), sizeof(g));
    (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cnt), sizeof(c));
    printf("rep %d rc %d rows %d flags %d: all four launches %.1f us; block 0 of kl_main, totals over tiles (us):", rep, rc, rows, a.flags, ms * 1000);
    double tot = 0;
    for (int k = 1; k < 8; ++k) { printf(" [%s] %.1f", names[k], g[k] * 0.01); tot += g[k] * 0.01; }
    printf("  sum %.1f; stats kernel block 0: %.1f\n", tot, (g[9] + g[10] + g[11]) * 0.01);
  }
  return 0;
}
