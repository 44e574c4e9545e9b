// D2 softmax + KL regulariser (model.py:98, train.py:85 'kullback_leibler_divergence'),
// TF-Adam (train.py:84 'adam' -> ResourceApplyAdam) and the device step counter.
#include "common.hpp"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float block_reduce(float v, float *red, bool is_max) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float o = __shfl_xor(v, off);
    v = is_max ? fmaxf(v, o) : v + o;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
  for (int w = 1; w < NT / 64; ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
  return r;
}

__device__ __forceinline__ double block_reduce_d(double v, double *red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = red[0];
  for (int w = 1; w < NT / 64; ++w) r += red[w];
  return r;
}

// One workgroup per regulariser row b.  p = softmax(z2[b]); t = clip(M~[reg_idx[b]], 1e-7, 1);
// q = clip(p, 1e-7, 1); KL_b = sum t log(t/q).  Gradient (TF clip_by_value = Minimum/Maximum
// grads: passes where p >= 1e-7): g_j = -t_j/p_j [p_j >= 1e-7]; <p,g> = -S, S = sum_{p>=1e-7} t;
// dz_j = reg/B * (p_j g_j + p_j S) = reg/B * ([p_j>=1e-7] (-t_j) + p_j S).
template <typename T>
__global__ __launch_bounds__(NT) void softmax_kl_kernel(const float *__restrict__ Z2, int V,
                                                        const float *__restrict__ Mt,
                                                        const int32_t *__restrict__ reg_idx,
                                                        float scale, T *__restrict__ dZ,
                                                        double *__restrict__ kl_part) {
  __shared__ float redf[NT / 64];
  __shared__ double redd[NT / 64];
  const int b = blockIdx.x;
  const float *z = Z2 + (int64_t)b * V;
  const float *trow = Mt + (int64_t)reg_idx[b] * V;
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < V; j += NT) mx = fmaxf(mx, z[j]);
  mx = block_reduce(mx, redf, true);
  float se = 0.f;
  for (int j = threadIdx.x; j < V; j += NT) se += expf(z[j] - mx);
  se = block_reduce(se, redf, false);
  const float inv = 1.f / se;
  double kl = 0.0, S = 0.0;
  for (int j = threadIdx.x; j < V; j += NT) {
    const float p = expf(z[j] - mx) * inv;
    const float t = fminf(fmaxf(trow[j], 1e-7f), 1.f);
    const float q = fminf(fmaxf(p, 1e-7f), 1.f);
    kl += (double)(t * logf(t / q));
    if (p >= 1e-7f) S += (double)t;
  }
  kl = block_reduce_d(kl, redd);
  S = block_reduce_d(S, redd);
  const float Sf = (float)S;
  for (int j = threadIdx.x; j < V; j += NT) {
    const float p = expf(z[j] - mx) * inv;
    const float t = fminf(fmaxf(trow[j], 1e-7f), 1.f);
    const float g = (p >= 1e-7f) ? -t : 0.f;
    DT<T>::st(dZ + (int64_t)b * V + j, scale * (g + p * Sf));
  }
  if (threadIdx.x == 0) kl_part[b] = kl;
}

// TF ResourceApplyAdam: alpha = lr sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
// p -= m*alpha/(sqrt(v)+eps).  t = state[0] + 1.
__global__ __launch_bounds__(NT) void adam_kernel(float *__restrict__ p, float *__restrict__ m,
                                                  float *__restrict__ v,
                                                  const float *__restrict__ g,
                                                  bf16_t *__restrict__ shadow, int64_t n,
                                                  const int64_t *__restrict__ state, float lr,
                                                  float b1, float b2, float eps) {
  const float t = (float)(state[0] + 1);
  const float b1p = powf(b1, t), b2p = powf(b2, t);
  const float alpha = lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float omb1 = 1.f - b1, omb2 = 1.f - b2;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4 *>(p)[i];
    float4 mm = reinterpret_cast<float4 *>(m)[i];
    float4 vv = reinterpret_cast<float4 *>(v)[i];
    const float4 gg = reinterpret_cast<const float4 *>(g)[i];
    float *pe = &pp.x, *me = &mm.x, *ve = &vv.x;
    const float *ge = &gg.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      me[e] += (ge[e] - me[e]) * omb1;
      ve[e] += (ge[e] * ge[e] - ve[e]) * omb2;
      pe[e] -= (me[e] * alpha) / (sqrtf(ve[e]) + eps);
    }
    reinterpret_cast<float4 *>(p)[i] = pp;
    reinterpret_cast<float4 *>(m)[i] = mm;
    reinterpret_cast<float4 *>(v)[i] = vv;
    if (shadow) {
      ushort4 s;
      s.x = f2bf(pp.x);
      s.y = f2bf(pp.y);
      s.z = f2bf(pp.z);
      s.w = f2bf(pp.w);
      reinterpret_cast<ushort4 *>(shadow)[i] = s;
    }
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    m[i] += (g[i] - m[i]) * omb1;
    v[i] += (g[i] * g[i] - v[i]) * omb2;
    p[i] -= (m[i] * alpha) / (sqrtf(v[i]) + eps);
    if (shadow) shadow[i] = f2bf(p[i]);
  }
}

__global__ void state_advance_kernel(int64_t *state, int64_t bpe) {
  state[0] += 1;
  state[1] += 1;
  if (state[1] >= bpe) {
    state[1] = 0;
    state[2] += 1;
  }
}

__global__ __launch_bounds__(NT) void to_bf16_kernel(const float *__restrict__ x,
                                                     bf16_t *__restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = f2bf(x[i]);
}

}  // namespace

extern "C" int cc_dec_softmax_kl_fused(int32_t dtype, const float *Z2, int32_t B, int32_t V,
                                       const float *y_reg, const int32_t *reg_idx, float reg,
                                       void *dZ, double *kl_partials, void *stream) {
  CC_REQUIRE(Z2 && y_reg && reg_idx && dZ && kl_partials, "cc_dec_softmax_kl_fused: null pointer");
  if (B == 0) return CC_OK;
  const float scale = reg / (float)B;
  if (dtype == CC_BF16)
    hipLaunchKernelGGL(softmax_kl_kernel<bf16_t>, dim3(B), dim3(NT), 0, as_stream(stream), Z2, V,
                       y_reg, reg_idx, scale, (bf16_t *)dZ, kl_partials);
  else
    hipLaunchKernelGGL(softmax_kl_kernel<float>, dim3(B), dim3(NT), 0, as_stream(stream), Z2, V,
                       y_reg, reg_idx, scale, (float *)dZ, kl_partials);
  CC_LAUNCH_CHECK("softmax_kl_kernel");
  return CC_OK;
}

extern "C" int cc_adam_dense(float *p, float *m, float *v, const float *g, uint16_t *shadow,
                             int64_t n, const int64_t *state, float lr, float beta1, float beta2,
                             float eps, void *stream) {
  CC_REQUIRE(p && m && v && g && state, "cc_adam_dense: null pointer");
  CC_REQUIRE(((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g) % 16 == 0,
             "cc_adam_dense: buffers must be 16-byte aligned");
  CC_REQUIRE(!shadow || (uintptr_t)shadow % 8 == 0, "cc_adam_dense: shadow must be 8-byte aligned");
  if (n <= 0) return CC_OK;
  const int64_t blocks = std::min<int64_t>(cdiv(cdiv(n, 4), NT), 256 * 8);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(NT), 0, as_stream(stream), p, m, v,
                     g, (bf16_t *)shadow, n, state, lr, beta1, beta2, eps);
  CC_LAUNCH_CHECK("adam_kernel");
  return CC_OK;
}

extern "C" int cc_state_advance(int64_t *state, int64_t batches_per_epoch, void *stream) {
  CC_REQUIRE(state && batches_per_epoch >= 1, "cc_state_advance: args");
  hipLaunchKernelGGL(state_advance_kernel, dim3(1), dim3(1), 0, as_stream(stream), state,
                     batches_per_epoch);
  CC_LAUNCH_CHECK("state_advance_kernel");
  return CC_OK;
}

extern "C" int cc_to_bf16(const float *x, uint16_t *y, int64_t n, void *stream) {
  CC_REQUIRE(x && y, "cc_to_bf16: null");
  if (n <= 0) return CC_OK;
  const int64_t blocks = std::min<int64_t>(cdiv(n, NT), 2048);
  hipLaunchKernelGGL(to_bf16_kernel, dim3((unsigned)blocks), dim3(NT), 0, as_stream(stream), x,
                     (bf16_t *)y, n);
  CC_LAUNCH_CHECK("to_bf16_kernel");
  return CC_OK;
}
