// A/B of cc_dec_softmax_kl_dw's many-row paths: the default (flags 0) against cc_dec_kl_args.flags
// argv[2] (default: CC_KL_LDS_TARGETS | CC_KL_DWO_PRODUCER_WAVES) on random full-mode inputs; prints
// how many dZ / dWo / dbo elements and which losses differ, and the first differing dbo column.
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/kl_ab.hip \
//   cubecobrarecommender_amd/csrc/decreg.hip cubecobrarecommender_amd/csrc/api.cpp \
//   cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/gpubin/kl_ab
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ccrec.h"

static uint16_t bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

int main(int argc, char **argv) {
  const int V = argc > 1 ? atoi(argv[1]) : 2500, d = 256, B = 128;
  const int rows = (V + 31) / 32 * 32, R = B + rows;
  std::mt19937 g(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::uniform_real_distribution<float> ud(0.f, 1.f);
  std::vector<uint16_t> h3((size_t)R * d), hw((size_t)V * d);
  for (auto &x : h3) x = bf(0.5f * nd(g));
  for (auto &x : hw) x = bf(0.2f * nd(g));
  std::vector<float> hb(V), hm((size_t)V * V, 0.f);
  for (auto &x : hb) x = 0.5f * nd(g);
  for (auto &x : hm) x = ud(g) < 0.05f ? ud(g) : 0.f;
  std::vector<int> hr(rows);
  for (int i = 0; i < rows; ++i) hr[i] = i < V ? i : -1;
  void *D3p, *D3tp, *Wo, *bo, *Mt, *tsum, *ridx, *ws, *tick;
  (void)hipMalloc(&D3p, h3.size() * 2);
  (void)hipMalloc(&D3tp, h3.size() * 2);
  (void)hipMalloc(&Wo, hw.size() * 2);
  (void)hipMalloc(&bo, V * 4);
  (void)hipMalloc(&Mt, hm.size() * 4);
  (void)hipMalloc(&tsum, V * 8);
  (void)hipMalloc(&ridx, rows * 4);
  (void)hipMalloc(&ws, cc_dec_kl_ws_size(rows, V));
  (void)hipMalloc(&tick, 8);
  (void)hipMemcpy(D3p, h3.data(), h3.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(D3tp, h3.data(), h3.size() * 2, hipMemcpyHostToDevice);   // (any bits: a dWo A operand)
  (void)hipMemcpy(Wo, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(bo, hb.data(), V * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(Mt, hm.data(), hm.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(ridx, hr.data(), rows * 4, hipMemcpyHostToDevice);
  (void)hipMemset(tick, 0, 8);
  cc_kl_tsum((const float *)Mt, V, V, (float *)tsum, nullptr);
  struct Out { std::vector<uint16_t> dz; std::vector<float> gw, gb; double loss; };
  Out o[2];
  for (int f = 0; f < 2; ++f) {
    void *dZ, *gW, *gb, *part, *loss;
    (void)hipMalloc(&dZ, (size_t)rows * V * 2);
    (void)hipMalloc(&gW, (size_t)d * V * 4);
    (void)hipMalloc(&gb, V * 4);
    (void)hipMalloc(&part, 4096 * 8);
    (void)hipMalloc(&loss, 8);
    cc_dec_kl_args a{};
    a.d = d; a.V = V; a.rows = rows; a.ldt = R; a.row0 = B;
    a.D3p = D3p; a.D3tp = D3tp; a.Wo = Wo; a.bo = (const float *)bo; a.Mt = (const float *)Mt;
    a.tsum = (const float *)tsum; a.mt_bytes = (int64_t)V * V * 4; a.mt_lo = 0; a.reg_idx = (const int32_t *)ridx;
    a.scale = 1.f / rows; a.dZ = dZ; a.gW = (float *)gW; a.gb = (float *)gb; a.loss_partials = (double *)part;
    a.loss_out = (double *)loss; a.loss_scale = 1.0 / rows; a.ticket = (uint32_t *)tick; a.ws = ws;
    a.flags = f ? (argc > 2 ? atoi(argv[2]) : CC_KL_LDS_TARGETS | CC_KL_DWO_PRODUCER_WAVES) : 0;
    const int rc = cc_dec_softmax_kl_dw(&a, nullptr);
    (void)hipDeviceSynchronize();
    o[f].dz.resize((size_t)rows * V);
    o[f].gw.resize((size_t)d * V);
    o[f].gb.resize(V);
    (void)hipMemcpy(o[f].dz.data(), dZ, o[f].dz.size() * 2, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o[f].gw.data(), gW, o[f].gw.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o[f].gb.data(), gb, V * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&o[f].loss, loss, 8, hipMemcpyDeviceToHost);
    printf("flags %d rc %d loss %.17g\n", f, rc, o[f].loss);
  }
  size_t ndz = 0, ngw = 0, ngb = 0;
  for (size_t i = 0; i < o[0].dz.size(); ++i) ndz += o[0].dz[i] != o[1].dz[i];
  for (size_t i = 0; i < o[0].gw.size(); ++i) ngw += std::memcmp(&o[0].gw[i], &o[1].gw[i], 4) != 0;
  int first = -1;
  for (int i = 0; i < V; ++i)
    if (std::memcmp(&o[0].gb[i], &o[1].gb[i], 4) != 0) {
      ++ngb;
      if (first < 0) first = i;
    }
  // FNV-1a over the default path's outputs: equal across two builds = the same bits
  uint64_t h = 1469598103934665603ull;
  auto fnv = [&](const void *p, size_t n) {
    const unsigned char *c = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  };
  fnv(o[0].dz.data(), o[0].dz.size() * 2);
  fnv(o[0].gw.data(), o[0].gw.size() * 4);
  fnv(o[0].gb.data(), o[0].gb.size() * 4);
  fnv(&o[0].loss, 8);
  printf("default-path outputs hash %016llx\n", (unsigned long long)h);
  printf("V %d rows %d: differing dZ %zu, dWo %zu, dbo %zu", V, rows, ndz, ngw, ngb);
  if (first >= 0) printf(" (first dbo column %d: %.9g vs %.9g, slice %d)", first, o[0].gb[first], o[1].gb[first], first / 96);
  printf("\n");
  return 0;
}
