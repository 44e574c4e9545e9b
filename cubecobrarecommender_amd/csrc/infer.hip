// Recommend forward pass in fp32 with a PINNED summation order — bit-exact against
// oracle/infer_ref.py.  Replaces `model.encoder(x)` / `model.decoder(z)` of
// src/scripts/ml_recommend.py:78-85 and web/ml_recommend_web.py:39-44.
//
// Pinned arithmetic (every multiply and add separately rounded: contraction is off here):
//   E1:   sorted unique card ids in chunks of 32; each chunk summed from 0 in order; chunk sums
//         added in order from 0; + bias; ReLU = (x > 0 ? x : 0).
//   Dense: K in chunks of 64; chunk acc = acc + h[k]*W[k][c] from 0; chunk partials added in
//          order from 0; + bias; ReLU.
//   Output: same dot, then sigmoid = float(1/(1+exp(-z))) in fp64 with the deterministic exp.
// tower_kernel: one workgroup per cube row, activations in LDS; out_kernel: one thread per card.
#include "common.hpp"
#include "detmath.hpp"

namespace {

constexpr int NT = 512;
constexpr int GCH = 32;   // gather chunk (rows)
constexpr int GGRP = 16;  // chunks per LDS group
constexpr int KCH = 64;   // dot chunk

struct Layer {
  const float *W, *b;
  int K, N;
};
struct Tower {
  const float *W1, *b1;  // E1 (gather)
  Layer L[3];
  int d;
};

__device__ __forceinline__ float addf(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float mulf(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// out[n] = relu?(blocked_dot(h, W[:, n]) + b[n]); scratch = [K/KCH][N] floats
__device__ void dense_lds(const float *h, const Layer &L, float *out, float *scratch, bool do_relu) {
  const int nch = (L.K + KCH - 1) / KCH;
  for (int t = threadIdx.x; t < nch * L.N; t += NT) {
    const int c = t / L.N, n = t % L.N;
    const int k0 = c * KCH, k1 = min(L.K, k0 + KCH);
    float acc = 0.f;
    for (int k = k0; k < k1; ++k) acc = addf(acc, mulf(h[k], L.W[(int64_t)k * L.N + n]));
    scratch[t] = acc;
  }
  __syncthreads();
  for (int n = threadIdx.x; n < L.N; n += NT) {
    float tot = 0.f;
    for (int c = 0; c < nch; ++c) tot = addf(tot, scratch[c * L.N + n]);
    const float v = addf(tot, L.b[n]);
    out[n] = do_relu ? relu(v) : v;
  }
  __syncthreads();
}

// mode 0: encode (gather + e2,e3,bottleneck) -> zlat[R,64]
// mode 1: decode tower (d1,d2,d3) from zlat -> h3[R,d]
__global__ __launch_bounds__(NT) void tower_kernel(Tower T, int mode, const int32_t *row_ptr,
                                                   const int32_t *idx, const float *zin,
                                                   float *out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int d = T.d;
  float *hA = sm;                // [max(d,256)]
  float *hB = hA + 1024;         // [1024]
  float *scratch = hB + 1024;    // [max(GGRP*d, K/KCH*N)]
  const int r = blockIdx.x;
  if (mode == 0) {
    const int beg = row_ptr[r], n = row_ptr[r + 1] - beg;
    const int32_t *lst = idx + beg;
    for (int c = threadIdx.x; c < d; c += NT) hB[c] = 0.f;  // running total
    const int nchunks = (n + GCH - 1) / GCH;
    for (int g0 = 0; g0 < nchunks; g0 += GGRP) {
      const int gcnt = min(GGRP, nchunks - g0);
      __syncthreads();
      for (int t = threadIdx.x; t < gcnt * d; t += NT) {
        const int c = t / d, col = t % d;
        const int j0 = (g0 + c) * GCH, j1 = min(n, j0 + GCH);
        float acc = 0.f;
        for (int j = j0; j < j1; ++j) acc = addf(acc, T.W1[(int64_t)lst[j] * d + col]);
        scratch[t] = acc;
      }
      __syncthreads();
      for (int col = threadIdx.x; col < d; col += NT) {
        float tot = hB[col];
        for (int c = 0; c < gcnt; ++c) tot = addf(tot, scratch[c * d + col]);
        hB[col] = tot;
      }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < d; col += NT) hA[col] = relu(addf(hB[col], T.b1[col]));
    __syncthreads();
  } else {
    for (int c = threadIdx.x; c < 64; c += NT) hA[c] = zin[(int64_t)r * 64 + c];
    __syncthreads();
  }
  dense_lds(hA, T.L[0], hB, scratch, true);
  dense_lds(hB, T.L[1], hA, scratch, true);
  dense_lds(hA, T.L[2], hB, scratch, true);
  const int N = T.L[2].N;
  for (int c = threadIdx.x; c < N; c += NT) out[(int64_t)r * N + c] = hB[c];
}

__global__ __launch_bounds__(256) void out_kernel(const float *__restrict__ h3, const float *Wo,
                                                  const float *bo, int d, int V,
                                                  float *__restrict__ probs) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = blockIdx.y;
  if (n >= V) return;
  const float *h = h3 + (int64_t)r * d;
  float tot = 0.f;
  for (int k0 = 0; k0 < d; k0 += KCH) {
    const int k1 = min(d, k0 + KCH);
    float acc = 0.f;
    for (int k = k0; k < k1; ++k) acc = addf(acc, mulf(h[k], Wo[(int64_t)k * V + n]));
    tot = addf(tot, acc);
  }
  probs[(int64_t)r * V + n] = detm::det_sigmoid32(addf(tot, bo[n]));
}

int tower_lds_bytes(int d) {
  int scratch = GGRP * d;
  const int shapes[6][2] = {{d, 256}, {256, 128}, {128, 64}, {64, 128}, {128, 256}, {256, d}};
  for (auto &s : shapes) scratch = std::max(scratch, ((s[0] + KCH - 1) / KCH) * s[1]);
  return (2048 + scratch) * 4;
}

}  // namespace

// layout helper implemented in api.cpp
namespace cc {
int param_offsets(int V, int d, int64_t *off, int64_t *size, int64_t *total, int64_t *main_total);
}

static int make_tower(const float *params, int V, int d, bool encoder, Tower &T) {
  int64_t off[CC_NUM_TENSORS], sz[CC_NUM_TENSORS], tot, mt;
  int rc = cc::param_offsets(V, d, off, sz, &tot, &mt);
  if (rc) return rc;
  T.d = d;
  const int base = encoder ? 0 : 8;  // tensor index of first kernel (e1 or decoder/d1)
  const int Ks[2][3] = {{d, 256, 128}, {64, 128, 256}};
  const int Ns[2][3] = {{256, 128, 64}, {128, 256, d}};
  const int e = encoder ? 0 : 1;
  if (encoder) {
    T.W1 = params + off[0];
    T.b1 = params + off[1];
  } else {
    T.W1 = nullptr;
    T.b1 = nullptr;
  }
  for (int l = 0; l < 3; ++l) {
    const int ti = encoder ? 2 + 2 * l : base + 2 * l;
    T.L[l].W = params + off[ti];
    T.L[l].b = params + off[ti + 1];
    T.L[l].K = Ks[e][l];
    T.L[l].N = Ns[e][l];
  }
  return CC_OK;
}

extern "C" int cc_infer_encode_fp32(const float *params, int32_t V, int32_t d, int32_t R,
                                    const int32_t *row_ptr, const int32_t *idx, float *zlat,
                                    void *stream) {
  CC_REQUIRE(params && row_ptr && idx && zlat, "cc_infer_encode_fp32: null pointer");
  CC_REQUIRE(d >= 64 && d <= 1024 && d % 64 == 0, "cc_infer_encode_fp32: d");
  if (R == 0) return CC_OK;
  Tower T;
  int rc = make_tower(params, V, d, true, T);
  if (rc) return rc;
  hipLaunchKernelGGL(tower_kernel, dim3(R), dim3(NT), tower_lds_bytes(d), as_stream(stream), T, 0,
                     row_ptr, idx, (const float *)nullptr, zlat);
  CC_LAUNCH_CHECK("tower_kernel(encode)");
  return CC_OK;
}

extern "C" int cc_infer_decode_fp32(const float *params, int32_t V, int32_t d, int32_t R,
                                    const float *zlat, float *h3_ws, float *probs, void *stream) {
  CC_REQUIRE(params && zlat && h3_ws && probs, "cc_infer_decode_fp32: null pointer");
  CC_REQUIRE(d >= 64 && d <= 1024 && d % 64 == 0, "cc_infer_decode_fp32: d");
  if (R == 0) return CC_OK;
  Tower T;
  int rc = make_tower(params, V, d, false, T);
  if (rc) return rc;
  hipLaunchKernelGGL(tower_kernel, dim3(R), dim3(NT), tower_lds_bytes(d), as_stream(stream), T, 1,
                     (const int32_t *)nullptr, (const int32_t *)nullptr, zlat, h3_ws);
  CC_LAUNCH_CHECK("tower_kernel(decode)");
  int64_t off[CC_NUM_TENSORS], sz[CC_NUM_TENSORS], tot, mt;
  rc = cc::param_offsets(V, d, off, sz, &tot, &mt);
  if (rc) return rc;
  hipLaunchKernelGGL(out_kernel, dim3((unsigned)cdiv(V, 256), R), dim3(256), 0, as_stream(stream),
                     h3_ws, params + off[14], params + off[15], d, V, probs);
  CC_LAUNCH_CHECK("out_kernel");
  return CC_OK;
}
