// Adam loop-shape microbenchmark at the bench parameter count (dev tool):
// U float4 groups per thread per iteration (loads hoisted), optional non-temporal hints, grid size.
// hipcc -O3 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc tools/micro/adam_variants.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "adam.hpp"

typedef float f4v __attribute__((ext_vector_type(4)));

template <int U, bool NTMP>
__global__ __launch_bounds__(256) void adam_u(float *__restrict__ p, float *__restrict__ m,
                                              float *__restrict__ v, const float *__restrict__ g,
                                              bf16_t *__restrict__ sh, int64_t n4, float alpha) {
  const float omb1 = 0.1f, omb2 = 0.001f, eps = 1e-7f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; i0 < n4; i0 += stride) {
    f4v P[U], M[U], Vv[U], G[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < n4) {
        if (NTMP) {
          P[u] = __builtin_nontemporal_load(reinterpret_cast<f4v *>(p) + i);
          M[u] = __builtin_nontemporal_load(reinterpret_cast<f4v *>(m) + i);
          Vv[u] = __builtin_nontemporal_load(reinterpret_cast<f4v *>(v) + i);
          G[u] = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(g) + i);
        } else {
          P[u] = reinterpret_cast<f4v *>(p)[i];
          M[u] = reinterpret_cast<f4v *>(m)[i];
          Vv[u] = reinterpret_cast<f4v *>(v)[i];
          G[u] = reinterpret_cast<const f4v *>(g)[i];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i >= n4) continue;
      #pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = P[u][e], me = M[u][e], ve = Vv[u][e];
        cc_adam::elem(pe, me, ve, G[u][e], alpha, omb1, omb2, eps);
        P[u][e] = pe; M[u][e] = me; Vv[u][e] = ve;
      }
      ushort4 s;
      s.x = f2bf(P[u][0]);
      s.y = f2bf(P[u][1]);
      s.z = f2bf(P[u][2]);
      s.w = f2bf(P[u][3]);
      if (NTMP) {
        __builtin_nontemporal_store(P[u], reinterpret_cast<f4v *>(p) + i);
        __builtin_nontemporal_store(M[u], reinterpret_cast<f4v *>(m) + i);
        __builtin_nontemporal_store(Vv[u], reinterpret_cast<f4v *>(v) + i);
      } else {
        reinterpret_cast<f4v *>(p)[i] = P[u];
        reinterpret_cast<f4v *>(m)[i] = M[u];
        reinterpret_cast<f4v *>(v)[i] = Vv[u];
      }
      reinterpret_cast<ushort4 *>(sh)[i] = s;
    }
  }
}

template <int U, bool NTMP>
void run(const char *name, float *p, float *m, float *v, float *g, bf16_t *sh, int64_t n4, int grid) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((adam_u<U, NTMP>), dim3(grid), dim3(256), 0, 0, p, m, v, g, sh, n4, 1e-9f);
  (void)hipEventRecord(a);
  const int reps = 50;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((adam_u<U, NTMP>), dim3(grid), dim3(256), 0, 0, p, m, v, g, sh, n4, 1e-9f);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / reps, bytes = n4 * 4.0 * 30.0;
  printf("%-10s U=%d nt=%d grid=%5d: %6.1f us  %6.0f GB/s\n", name, U, (int)NTMP, grid, us, bytes / us / 1e3);
}

int main() {
  const int64_t n = 11520000, n4 = n / 4;
  float *p, *m, *v, *g;
  bf16_t *sh;
  (void)hipMalloc(&p, n * 4);
  (void)hipMalloc(&m, n * 4);
  (void)hipMalloc(&v, n * 4);
  (void)hipMalloc(&g, n * 4);
  (void)hipMalloc(&sh, n * 2);
  (void)hipMemset(p, 0, n * 4);
  (void)hipMemset(m, 0, n * 4);
  (void)hipMemset(v, 0, n * 4);
  (void)hipMemset(g, 0, n * 4);
  for (int grid : {1024, 2048, 4096}) {
    run<1, false>("base", p, m, v, g, sh, n4, grid);
    run<2, false>("u2", p, m, v, g, sh, n4, grid);
    run<4, false>("u4", p, m, v, g, sh, n4, grid);
    run<1, true>("nt", p, m, v, g, sh, n4, grid);
    run<2, true>("u2nt", p, m, v, g, sh, n4, grid);
    run<4, true>("u4nt", p, m, v, g, sh, n4, grid);
  }
  const int64_t full = (n4 + 255) / 256;
  run<1, false>("onepass", p, m, v, g, sh, n4, (int)full);
  run<1, true>("onepassnt", p, m, v, g, sh, n4, (int)full);
  run<2, true>("halfnt", p, m, v, g, sh, n4, (int)((full + 1) / 2));
  printf("err %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
