// Per-wave end times of embed_grad_cs_kernel's REG + Adam instance (cc_embed_grad_cs_adam_reg) at
// V = 22,000, d = 256, B = 512 cube rows + 512 reg rows by index, with and without the bias row
// (dev tool): which wave of which block ends the launch.  Lane 0 of every wave stamps
// s_memrealtime (10 ns) at the kernel's probe points (EG_PROBE: 0 start, 1 staged, 2 barrier,
// 3 tiles done, 15 end).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/eg_reg_probe.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/gpubin/eg_reg_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

__device__ unsigned long long g_probe[1024][5][8];
#define EG_PROBE(k)                                                                                          \
  do {                                                                                                       \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                                                        \
      g_probe[blockIdx.x][(k) == 15 ? 4 : ((k) > 3 ? 3 : (k))][threadIdx.x >> 6] = wall_clock64();          \
  } while (0)
#include "embed.hip"

// (the gather entry point in embed.hip references it; not called here)
extern "C" int cc_state_advance(int64_t *, int64_t, void *) { return 0; }

int main() {
  const int V = 22000, d = 256, B = 512, RP = 1024, nreg = 512;
  void *gP, *xt, *bg, *tk, *p, *m, *v, *sh, *st, *rid;
  (void)hipMalloc(&gP, (size_t)d * RP * 2);
  (void)hipMalloc(&xt, (size_t)V * (B / 32) * 4);
  (void)hipMalloc(&bg, d * 4);
  (void)hipMalloc(&tk, 4096 * 4);
  (void)hipMalloc(&p, (size_t)V * d * 4);
  (void)hipMalloc(&m, (size_t)V * d * 4);
  (void)hipMalloc(&v, (size_t)V * d * 4);
  (void)hipMalloc(&sh, (size_t)V * d * 2);
  (void)hipMalloc(&st, 4 * 8);
  (void)hipMalloc(&rid, nreg * 4);
  (void)hipMemset(gP, 0, (size_t)d * RP * 2);
  (void)hipMemset(p, 0, (size_t)V * d * 4);
  (void)hipMemset(m, 0, (size_t)V * d * 4);
  (void)hipMemset(v, 0, (size_t)V * d * 4);
  (void)hipMemset(st, 0, 32);
  (void)hipMemset(tk, 0, 4096 * 4);
  std::vector<uint32_t> bits((size_t)V * (B / 32));
  uint32_t x = 12345;
  for (auto &b : bits) {
    uint32_t w = 0;
    for (int i = 0; i < 32; ++i) { x = x * 1664525u + 1013904223u; if ((x >> 8) % 50 == 0) w |= 1u << i; }
    b = w;
  }
  (void)hipMemcpy(xt, bits.data(), bits.size() * 4, hipMemcpyHostToDevice);
  // reg cards: Zipf-like popularity (the bench's neg_sampler is popularity-weighted)
  std::vector<double> cdf(V);
  double s = 0;
  for (int i = 0; i < V; ++i) cdf[i] = (s += 1.0 / std::pow(i + 1.0, 0.9));
  std::vector<int32_t> r(nreg);
  for (int i = 0; i < nreg; ++i) {
    x = x * 1664525u + 1013904223u;
    const double u = (x >> 8) / 16777216.0 * s;
    r[i] = (int32_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
  }
  (void)hipMemcpy(rid, r.data(), nreg * 4, hipMemcpyHostToDevice);
  const int nsl = d / 32, nblk = cc_embed_grad_cs_tickets(V, d, B) * nsl;
  for (int rep = 0; rep < 6; ++rep) {
    const bool bias = rep & 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    const int rc = cc_embed_grad_cs_adam_reg(gP, 1, V, d, B, RP, (uint32_t *)xt, bias ? (float *)bg : nullptr, nullptr,
                                             (float *)p, (float *)m, (float *)v, (uint16_t *)sh, (const int64_t *)st,
                                             1e-3f, 0.9f, 0.999f, 1e-7f, (const int32_t *)rid, nreg, B / 16, nullptr);
    (void)hipEventRecord(b);
    (void)hipDeviceSynchronize();
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    static unsigned long long h[1024][5][8];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_probe), sizeof(h));
    unsigned long long t0 = ~0ull;
    for (int i = 0; i < nblk; ++i) t0 = std::min(t0, h[i][0][0]);
    // the latest-ending blocks and, in each, every wave's tile-loop end
    std::vector<std::pair<double, int>> ends;
    for (int i = 0; i < nblk; ++i) {
      unsigned long long e = 0;
      for (int w = 0; w < 8; ++w) e = std::max(e, h[i][4][w]);
      ends.push_back({(e - t0) * 0.01, i});
    }
    std::sort(ends.rbegin(), ends.rend());
    double med = ends[ends.size() / 2].first;
    printf("rep %d bias %d rc %d: %.1f us (event), %d blocks; block end us: max %.2f median %.2f\n", rep, (int)bias, rc,
           ms * 1000, nblk, ends[0].first, med);
    for (int j = 0; j < 4; ++j) {
      const int i = ends[j].second;
      printf("   block %4d (chunk %d slice %d) start %.2f staged %.2f; wave tile-loop ends:", i, i / nsl, i % nsl,
             (h[i][0][0] - t0) * 0.01, (h[i][2][0] - t0) * 0.01);
      for (int w = 0; w < 8; ++w) printf(" %.2f", (h[i][3][w] - t0) * 0.01);
      printf("\n");
    }
  }
  return 0;
}
