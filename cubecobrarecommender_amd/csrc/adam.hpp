// TF ResourceApplyAdam element update and its flat-range loop, shared by the plain Adam kernel
// (loss_adam.hip) and the Adam + next-step-F kernel (noise.hip).
//   alpha = lr sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
//   p -= m*alpha/(sqrt(v)+eps);  t = state[0] + 1.
#pragma once
// build knob (A/B builds): the dense Adam's p / m / v / g streams non-temporal (1) or default (0);
// measured (r05zm): default policy 149.7 -> 164.8-167.2 us/step (BCE), 961 -> 1,020 (config 5)
#ifndef ADAM_NT
#define ADAM_NT 1
#endif
#include "common.hpp"

template <typename T>
__device__ __forceinline__ T ADAM_LD(const T *p) {
  if constexpr (ADAM_NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T>
__device__ __forceinline__ void ADAM_ST(T v, T *p) {
  if constexpr (ADAM_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

namespace cc_adam {

typedef __attribute__((ext_vector_type(4))) float f32x4_t;

__device__ __forceinline__ void elem(float &p, float &m, float &v, float g, float alpha,
                                     float omb1, float omb2, float eps) {
#pragma clang fp contract(off)  // every kernel that inlines this rounds identically (no FMA choice)
  m += (g - m) * omb1;
  v += (g * g - v) * omb2;
  p -= (m * alpha) / (sqrtf(v) + eps);
}

struct Args {
  float *p, *m, *v;
  const float *g;
  bf16_t *shadow;
  int64_t n;
  float lr, b1, b2, eps;
  int64_t eoff;  // element offset of p from the base the Pack's layer offsets count from
};

// Fragment-packed tower images (cc_adam_pack): the bf16 values of float4 group e..e+3 (one row
// k, columns n..n+3 of layer l) go to the forward image (rows n, reduction k: 4 scattered 2-B
// stores) and the backward image (rows k, reduction n: one 8-B store).  Same element order as
// tower.hip's pack_off.
struct Pack {
  int n;
  int K[9], N[9];
  int64_t off[9];
  bf16_t *wpf[9], *wpb[9];
  int64_t lo, hi;  // [lo, hi) covers every packed layer
};
__device__ __forceinline__ int64_t frag_off(int t, int j, int lane, int red) {
  return (((int64_t)t * (red / 16) + j) * 64 + lane) * 8;
}
__device__ __forceinline__ void pack4(const Pack &pk, int64_t e, const bf16_t (&b)[4]) {
  if (e < pk.lo || e >= pk.hi) return;
  for (int l = 0; l < pk.n; ++l) {
    const int64_t o = e - pk.off[l];
    const int K = pk.K[l], N = pk.N[l];
    if (o < 0 || o >= (int64_t)K * N) continue;
    const int k = (int)(o / N), n = (int)(o % N);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nn = n + q;
      pk.wpf[l][frag_off(nn >> 5, k >> 4, (nn & 31) + 32 * ((k >> 3) & 1), K) + (k & 7)] = b[q];
    }
    const int64_t ob = frag_off(k >> 5, n >> 4, (k & 31) + 32 * ((n >> 3) & 1), N) + (n & 7);
    *reinterpret_cast<uint2 *>(pk.wpb[l] + ob) =
        make_uint2((uint32_t)b[0] | ((uint32_t)b[1] << 16), (uint32_t)b[2] | ((uint32_t)b[3] << 16));
    return;
  }
}

// Blocks [0, nblocks) of whatever grid run this cover [0, n) grid-stride (float4 body + tail).
__device__ __forceinline__ void range(const Args &a, int64_t step, int bid, int nblocks,
                                      const Pack *pk = nullptr) {
  const float t = (float)(step + 1);
  const float b1p = powf(a.b1, t), b2p = powf(a.b2, t);
  const float alpha = a.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float omb1 = 1.f - a.b1, omb2 = 1.f - a.b2;
  const int64_t n4 = a.n >> 2;
  const int64_t stride = (int64_t)nblocks * blockDim.x;
  for (int64_t i = (int64_t)bid * blockDim.x + threadIdx.x; i < n4; i += stride) {
    // p, m, v, g stream through once per step: non-temporal loads and stores (the bf16 shadow and
    // the packed images, which the next step's kernels read, keep the default policy).  Measured
    // in the step: 180-184 -> 178 us (Adam -1.5 us; the next W1-gradient kernel -2.5 us: Adam no
    // longer evicts the lines it reads)
    f32x4_t pv = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.p) + i);
    f32x4_t mv = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.m) + i);
    f32x4_t vv4 = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.v) + i);
    const f32x4_t gv = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.g) + i);
    float4 pp = make_float4(pv[0], pv[1], pv[2], pv[3]), mm = make_float4(mv[0], mv[1], mv[2], mv[3]);
    float4 vv = make_float4(vv4[0], vv4[1], vv4[2], vv4[3]);
    const float4 gg = make_float4(gv[0], gv[1], gv[2], gv[3]);
    float *pe = &pp.x, *me = &mm.x, *ve = &vv.x;
    const float *ge = &gg.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) elem(pe[e], me[e], ve[e], ge[e], alpha, omb1, omb2, a.eps);
    ADAM_ST(f32x4_t{pp.x, pp.y, pp.z, pp.w}, reinterpret_cast<f32x4_t *>(a.p) + i);
    ADAM_ST(f32x4_t{mm.x, mm.y, mm.z, mm.w}, reinterpret_cast<f32x4_t *>(a.m) + i);
    ADAM_ST(f32x4_t{vv.x, vv.y, vv.z, vv.w}, reinterpret_cast<f32x4_t *>(a.v) + i);
    if (a.shadow) {
      ushort4 s;
      s.x = f2bf(pp.x);
      s.y = f2bf(pp.y);
      s.z = f2bf(pp.z);
      s.w = f2bf(pp.w);
      reinterpret_cast<ushort4 *>(a.shadow)[i] = s;
      if (pk) {
        const bf16_t b4[4] = {s.x, s.y, s.z, s.w};
        pack4(*pk, a.eoff + (i << 2), b4);
      }
    }
  }
  for (int64_t i = (n4 << 2) + (int64_t)bid * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    float pp = a.p[i], mm = a.m[i], vv = a.v[i];
    elem(pp, mm, vv, a.g[i], alpha, omb1, omb2, a.eps);
    a.p[i] = pp;
    a.m[i] = mm;
    a.v[i] = vv;
    if (a.shadow) a.shadow[i] = f2bf(pp);
  }
}

// range() for a few persistent blocks that share a launch with latency-bound work (the tower
// backward chains, tower.hip): U float4 groups per thread in flight before any is consumed, so a
// CU holding one such block still keeps enough bytes outstanding to stream.  Same element
// update and rounding as range(); no packed images.
template <int U>
__device__ __forceinline__ void range_u(const Args &a, int64_t step, int bid, int nblocks) {
  const float t = (float)(step + 1);
  const float b1p = powf(a.b1, t), b2p = powf(a.b2, t);
  const float alpha = a.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float omb1 = 1.f - a.b1, omb2 = 1.f - a.b2;
  const int64_t n4 = a.n >> 2;
  const int64_t stride = (int64_t)nblocks * blockDim.x;
  for (int64_t i0 = (int64_t)bid * blockDim.x + threadIdx.x; i0 < n4; i0 += U * stride) {
    f32x4_t pv[U], mv[U], vv[U], gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n4) {
        pv[u] = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.p) + i);
        mv[u] = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.m) + i);
        vv[u] = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.v) + i);
        gv[u] = ADAM_LD(reinterpret_cast<const f32x4_t *>(a.g) + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n4) break;
      float pe[4] = {pv[u][0], pv[u][1], pv[u][2], pv[u][3]};
      float me[4] = {mv[u][0], mv[u][1], mv[u][2], mv[u][3]};
      float ve[4] = {vv[u][0], vv[u][1], vv[u][2], vv[u][3]};
#pragma unroll
      for (int e = 0; e < 4; ++e) elem(pe[e], me[e], ve[e], gv[u][e], alpha, omb1, omb2, a.eps);
      ADAM_ST(f32x4_t{pe[0], pe[1], pe[2], pe[3]}, reinterpret_cast<f32x4_t *>(a.p) + i);
      ADAM_ST(f32x4_t{me[0], me[1], me[2], me[3]}, reinterpret_cast<f32x4_t *>(a.m) + i);
      ADAM_ST(f32x4_t{ve[0], ve[1], ve[2], ve[3]}, reinterpret_cast<f32x4_t *>(a.v) + i);
      if (a.shadow) {
        ushort4 s;
        s.x = f2bf(pe[0]);
        s.y = f2bf(pe[1]);
        s.z = f2bf(pe[2]);
        s.w = f2bf(pe[3]);
        reinterpret_cast<ushort4 *>(a.shadow)[i] = s;
      }
    }
  }
  for (int64_t i = (n4 << 2) + (int64_t)bid * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    float pp = a.p[i], mm = a.m[i], vv = a.v[i];
    elem(pp, mm, vv, a.g[i], alpha, omb1, omb2, a.eps);
    a.p[i] = pp;
    a.m[i] = mm;
    a.v[i] = vv;
    if (a.shadow) a.shadow[i] = f2bf(pp);
  }
}

}  // namespace cc_adam
