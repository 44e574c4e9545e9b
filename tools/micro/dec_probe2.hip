// Per-block phase timestamps of dec_bce_dw_kernel at the bench shape (B = 512, d = 256, V = 22000, Wo read
// in place, packed D3 images) on random operands (dev tool): HIP-event time of the call, start / end spread
// over blocks and per-phase medians.
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-honor-nans -I include -I cubecobrarecommender_amd/csrc [-DPROBE_OFF] [-D<knob>=...] tools/micro/dec_probe2.hip \
//   cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/dec_probe2
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__device__ unsigned long long g_blk[1024][16];
__device__ unsigned long long g_wav[1024][8][16];
#ifdef PROBE_OFF   // clean timing: the kernel exactly as the library builds it
#define DEC_PROBE(k)
#else
#define DEC_PROBE(k)                                                          \
  do {                                                                        \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_blk[blockIdx.x][(k)] = wall_clock64(); \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) g_wav[blockIdx.x][threadIdx.x >> 6][(k)] = wall_clock64(); \
  } while (0)
#endif
#ifndef DEC_SRC
#define DEC_SRC "decout.hip"
#endif
#include DEC_SRC

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

int main() {
  const int B = 512, d = 256, V = 22000, VW = (V + 31) / 32;
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
  void *D3 = upload_bf((size_t)B * d, 0.5f), *D3t = upload_bf((size_t)B * d, 0.5f);
  void *D3p = upload_bf((size_t)B * d, 0.5f), *D3tp = upload_bf((size_t)B * d, 0.5f);
  void *Wo = upload_bf((size_t)V * d, 0.05f);
  void *bo, *yb, *dZ, *gW, *gb, *part, *loss, *tick;
  (void)hipMalloc(&bo, V * 4);
  (void)hipMemset(bo, 0, V * 4);
  (void)hipMalloc(&yb, (size_t)B * VW * 4);
  void *yi;   // the target-mask image (cc_tower_args.y_img): the trainer's call, cc_dec_bce_dw_img
  (void)hipMalloc(&yi, (size_t)B * VW * 4);
  {
    std::vector<uint32_t> y((size_t)B * VW), img((size_t)B * VW);
    for (auto &x : y) x = (rng() & rng() & rng() & rng() & rng()) ;  // ~3 % ones
    for (int w = 0; w < VW; ++w)
      for (int r = 0; r < B; ++r) {
        const int pos = r & 31, row = (r & ~31) + 8 * (pos >> 3) + 4 * (pos & 1) + ((pos >> 1) & 3);
        img[(size_t)w * B + r] = y[(size_t)row * VW + w];
      }
    (void)hipMemcpy(yb, y.data(), y.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(yi, img.data(), img.size() * 4, hipMemcpyHostToDevice);
  }
  (void)hipMalloc(&dZ, (size_t)B * V * 2);
  (void)hipMalloc(&gW, (size_t)d * V * 4);
  (void)hipMalloc(&gb, V * 4);
  (void)hipMalloc(&part, 4096 * 8);
  (void)hipMalloc(&loss, 8);
  (void)hipMalloc(&tick, 8);
  (void)hipMemset(tick, 0, 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int nb = (V + 95) / 96;
#ifdef PROBE_OFF
  {
    std::vector<float> ts;
    for (int rep = 0; rep < 200; ++rep) {
      (void)hipEventRecord(e0, nullptr);
      cc_dec_bce_dw_img(D3, D3t, B, D3p, D3tp, nullptr, Wo, (const float *)bo, B, d, V, (const uint32_t *)yb,
                        (const uint32_t *)yi, dZ, V, (float *)gW, (float *)gb, (double *)part, (double *)loss,
                        1.0 / (B * V), (uint32_t *)tick, nullptr);
      (void)hipEventRecord(e1, nullptr);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 20) ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    printf("clean call us: min %.2f p25 %.2f median %.2f p75 %.2f\n", ts[0], ts[ts.size() / 4], ts[ts.size() / 2],
           ts[3 * ts.size() / 4]);
    return 0;
  }
#endif
  for (int rep = 0; rep < 6; ++rep) {
    (void)hipEventRecord(e0, nullptr);
    int rc = cc_dec_bce_dw_img(D3, D3t, B, D3p, D3tp, nullptr, Wo, (const float *)bo, B, d, V, (const uint32_t *)yb,
                               (const uint32_t *)yi, dZ, V, (float *)gW, (float *)gb, (double *)part, (double *)loss,
                               1.0 / (B * V), (uint32_t *)tick, nullptr);
    (void)hipEventRecord(e1, nullptr);
    (void)hipDeviceSynchronize();
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    static unsigned long long g[1024][16];
    (void)hipMemcpyFromSymbol(g, HIP_SYMBOL(g_blk), sizeof(g));
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < nb; ++b) t0 = std::min(t0, g[b][0]);
    std::vector<double> st, en, ph[9];
    for (int b = 0; b < nb; ++b) {
      st.push_back((g[b][0] - t0) * 10.0);
      en.push_back((g[b][8] - t0) * 10.0);
      for (int k = 1; k < 9; ++k) ph[k].push_back((g[b][k] - g[b][k - 1]) * 10.0);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    auto mx = [](const std::vector<double> &v) { return *std::max_element(v.begin(), v.end()); };
    printf("rep %d rc %d call %.1f us | blocks %d start max %.0f ns, end med %.0f max %.0f ns\n", rep, rc, ms * 1e3,
           nb, mx(st), med(en), mx(en));
    printf("   medians (ns): resident %.0f, p0 mfma %.0f, p0 epi %.0f, p1 mfma %.0f, p1 epi %.0f, sync %.0f, "
           "ph2 mfma %.0f, ph2 stores %.0f\n", med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]), med(ph[5]), med(ph[6]),
           med(ph[7]), med(ph[8]));
    if (rep == 5) {
      static unsigned long long gw[1024][8][16];
      (void)hipMemcpyFromSymbol(gw, HIP_SYMBOL(g_wav), sizeof(gw));
      for (int w = 0; w < 8; ++w) {
        std::vector<double> pt[9];
        for (int b = 0; b < nb; ++b)
          for (int k = 1; k < 9; ++k) pt[k].push_back((gw[b][w][k] - gw[b][0][0]) * 10.0);
        printf("   wave %d points (ns from block start, median): ", w);
        for (int k = 1; k < 9; ++k) printf("%.0f ", med(pt[k]));
        printf("\n");
      }
    }
  }
  return 0;
}
