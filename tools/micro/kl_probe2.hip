// Per-block phase timestamps of kl_main_kernel / kl_stats_kernel at the bench's +KL shape (512 regulariser
// rows, d = 256, V = 22000) on random operands (dev tool): start / end spread over blocks, per-phase medians,
// and HIP-event durations of the whole D2 call.
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/kl_probe2.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/kl_probe2
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

#ifndef PROBE_ROWS
#define PROBE_ROWS 512
#endif
__device__ unsigned long long g_main[1024][16];
__device__ unsigned long long g_stat[4096][16];
#define KL_PROBE(k)                                                                           \
  do {                                                                                        \
    if (threadIdx.x == 0) {                                                                   \
      if ((k) < 8) {                                                                          \
        if (sl < 1024) g_main[sl][(k)] = wall_clock64();                                      \
      } else if (blockIdx.x + gridDim.x * blockIdx.y < 4096) {                                \
        g_stat[blockIdx.x + gridDim.x * blockIdx.y][(k)-8] = wall_clock64();                 \
      }                                                                                       \
    }                                                                                         \
  } while (0)
#include "decreg.hip"

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

int main() {
  const int rows = PROBE_ROWS, B = 512, R = B + rows, d = 256, V = 22000;
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  auto upload_bf = [&](size_t n, float sd) {
    std::vector<uint16_t> h(n);
    for (auto &x : h) x = f2bf(sd * nd(rng));
    void *p;
    (void)hipMalloc(&p, n * 2);
    (void)hipMemcpy(p, h.data(), n * 2, hipMemcpyHostToDevice);
    return p;
  };
  void *D3p = upload_bf((size_t)R * d, 0.5f), *D3tp = upload_bf((size_t)R * d, 0.5f);
  void *Wo = upload_bf((size_t)V * d, 0.05f);
  void *bo, *Mt, *tsum, *ridx, *dZ, *gW, *gb, *part, *loss, *tick, *ws;
  (void)hipMalloc(&bo, V * 4);
  (void)hipMemset(bo, 0, V * 4);
  (void)hipMalloc(&Mt, (size_t)V * V * 4);
  {
    std::vector<float> row(V);
    std::uniform_real_distribution<float> u(0.f, 2.f / V);
    for (int r = 0; r < rows; ++r) {
      const int card = (r * 7919) % V;
      for (auto &x : row) x = u(rng);
      (void)hipMemcpy((float *)Mt + (size_t)card * V, row.data(), V * 4, hipMemcpyHostToDevice);
    }
  }
  (void)hipMalloc(&tsum, V * 4);
  {
    std::vector<float> t(V, 1.f);
    (void)hipMemcpy(tsum, t.data(), V * 4, hipMemcpyHostToDevice);
  }
  (void)hipMalloc(&ridx, rows * 4);
  (void)hipMalloc(&dZ, (size_t)rows * V * 2);
  (void)hipMalloc(&gW, (size_t)d * V * 4);
  (void)hipMalloc(&gb, V * 4);
  (void)hipMalloc(&part, 4096 * 8);
  (void)hipMalloc(&loss, 8);
  (void)hipMalloc(&tick, 8);
  (void)hipMemset(tick, 0, 8);
  (void)hipMalloc(&ws, cc_dec_kl_ws_size(rows, V));
  std::vector<int> h(rows);
  for (int i = 0; i < rows; ++i) h[i] = (i * 7919) % V;
  (void)hipMemcpy(ridx, h.data(), rows * 4, hipMemcpyHostToDevice);
  cc_dec_kl_args a{};
  a.d = d; a.V = V; a.rows = rows; a.ldt = R; a.row0 = B;
  a.D3p = D3p; a.D3tp = D3tp; a.Wo = Wo; a.bo = (const float *)bo; a.Mt = (const float *)Mt;
  a.tsum = (const float *)tsum; a.mt_bytes = std::min<int64_t>((int64_t)V * V * 4, 0x7FFFFFFF); a.mt_lo = 0;
  a.reg_idx = (const int32_t *)ridx;
  a.scale = 1e-4f; a.dZ = dZ; a.gW = (float *)gW; a.gb = (float *)gb; a.loss_partials = (double *)part;
  a.loss_out = (double *)loss; a.loss_scale = 1.0 / rows; a.ticket = (uint32_t *)tick; a.ws = ws;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int nsl = (V + 95) / 96;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, nullptr);
    int rc = cc_dec_softmax_kl_dw(&a, nullptr);
    (void)hipEventRecord(e1, nullptr);
    (void)hipDeviceSynchronize();
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    static unsigned long long gm[1024][16], gs[4096][16];
    (void)hipMemcpyFromSymbol(gm, HIP_SYMBOL(g_main), sizeof(gm));
    (void)hipMemcpyFromSymbol(gs, HIP_SYMBOL(g_stat), sizeof(gs));
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < nsl; ++b) t0 = std::min(t0, gm[b][0]);
    std::vector<double> st, en, ph[8];
    for (int b = 0; b < nsl; ++b) {
      st.push_back((gm[b][0] - t0) * 10.0);
      en.push_back((gm[b][7] - t0) * 10.0);
      for (int k = 1; k < 8; ++k) ph[k].push_back((gm[b][k] - gm[b][k - 1]) * 10.0);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    auto mx = [](const std::vector<double> &v) { return *std::max_element(v.begin(), v.end()); };
    printf("rep %d rc %d  call %.1f us | main blocks %d: start max %.0f ns, end med %.0f max %.0f ns\n", rep, rc,
           ms * 1e3, nsl, mx(st), med(en), mx(en));
    printf("   main phase medians (ns): staged %.0f, p0 logits %.0f, p0 epi %.0f, p1 logits %.0f, p1 epi %.0f, "
           "pre-ph2 %.0f, ph2+end %.0f\n", med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]), med(ph[5]), med(ph[6]),
           med(ph[7]));
    const int nb = nsl;  // probes fire in blockIdx.y == 0 only
    unsigned long long s0 = ~0ull;
    for (int b = 0; b < nb; ++b) s0 = std::min(s0, gs[b][0]);
    std::vector<double> ss, se, sp[4];
    for (int b = 0; b < nb; ++b) {
      ss.push_back((gs[b][0] - s0) * 10.0);
      se.push_back((gs[b][3] - s0) * 10.0);
      for (int k = 1; k < 4; ++k) sp[k].push_back((gs[b][k] - gs[b][k - 1]) * 10.0);
    }
    printf("   stats blocks %d: start max %.0f, end med %.0f max %.0f ns; phases (ns) staged %.0f logits+max %.0f "
           "reductions %.0f\n", nb, mx(ss), med(se), mx(se), med(sp[1]), med(sp[2]), med(sp[3]));
    printf("   stats start -> main start: %.0f ns\n", (double)(t0 - s0) * 10.0);
  }
  return 0;
}
