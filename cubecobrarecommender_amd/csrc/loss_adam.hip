// D2 softmax + KL regulariser (model.py:98, train.py:85 'kullback_leibler_divergence'),
// TF-Adam (train.py:84 'adam' -> ResourceApplyAdam) and the device step counter.
#include "adam.hpp"
#include "common.hpp"
#include "mx8.hpp"

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
// dz_j = scale * (p_j g_j + p_j S) = scale * ([p_j>=1e-7] (-t_j) + p_j S), scale = reg * the
// row's weight (1/B for B sampled rows).
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
  if (reg_idx[b] < 0) {  // padding row (owner-computes capacity): no KL term, zero gradient
    for (int j = threadIdx.x; j < V; j += NT) DT<T>::st(dZ + (int64_t)b * V + j, 0.f);
    if (threadIdx.x == 0) kl_part[b] = 0.0;
    return;
  }
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

// The same row computation with the row held in registers: one 1024-thread workgroup per row,
// z and t read from HBM exactly once as float4s (NV per thread, V <= 4096 NV), so the kernel
// moves 8 B/element in and sizeof(T) out — the HBM floor of the regulariser loss — instead of
// re-reading the row four times.  Same element formulas as softmax_kl_kernel.
constexpr int NTR = 1024;

template <typename Tv, int W>
__device__ __forceinline__ Tv rows_reduce(Tv v, Tv *red, bool is_max) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const Tv o = __shfl_xor(v, off);
    v = is_max ? (v > o ? v : o) : v + o;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  Tv r = red[0];
#pragma unroll
  for (int w = 1; w < W; ++w) r = is_max ? (r > red[w] ? r : red[w]) : r + red[w];
  return r;
}

// two fp64 sums reduced together (the same xor tree and wave order per value as rows_reduce: the
// same results, one barrier pair instead of two)
template <int W>
__device__ __forceinline__ void rows_reduce2(double &a, double &b, double *red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = a;
    red[W + (threadIdx.x >> 6)] = b;
  }
  __syncthreads();
  double ra = red[0], rb = red[W];
#pragma unroll
  for (int w = 1; w < W; ++w) {
    ra += red[w];
    rb += red[W + w];
  }
  a = ra;
  b = rb;
}

template <typename T, int NV>
__global__ __launch_bounds__(NTR) void softmax_kl_rows_kernel(const float *__restrict__ Z2, int V,
                                                              const float *__restrict__ Mt,
                                                              const int32_t *__restrict__ reg_idx,
                                                              float scale, T *__restrict__ dZ,
                                                              double *__restrict__ kl_part,
                                                              uint8_t *__restrict__ zq = nullptr, int ldzq = 0,
                                                              uint8_t *__restrict__ zqs = nullptr) {
  __shared__ float redf[NTR / 64];
  __shared__ double redd[2 * (NTR / 64)];
  const int b = blockIdx.x, V4 = V >> 2;
  if (reg_idx[b] < 0) {  // padding row (owner-computes capacity): no KL term, zero gradient
    for (int j = threadIdx.x; j < V; j += NTR) DT<T>::st(dZ + (int64_t)b * V + j, 0.f);
    if (zq) {            // zero codes, scale 2^0 (the quantiser's all-zero block)
      for (int j = threadIdx.x; j < ldzq / 4; j += NTR) reinterpret_cast<uint32_t *>(zq + (int64_t)b * ldzq)[j] = 0u;
      for (int j = threadIdx.x; j < ldzq / 32; j += NTR) zqs[(int64_t)b * (ldzq / 32) + j] = 127;
    }
    if (threadIdx.x == 0) kl_part[b] = 0.0;
    return;
  }
  const float4 *z4 = reinterpret_cast<const float4 *>(Z2 + (int64_t)b * V);
  const float4 *t4 = reinterpret_cast<const float4 *>(Mt + (int64_t)reg_idx[b] * V);
  float z[NV][4], t[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = threadIdx.x + i * NTR;
    const float4 zz = j < V4 ? z4[j] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    const float4 tt = j < V4 ? t4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    z[i][0] = zz.x, z[i][1] = zz.y, z[i][2] = zz.z, z[i][3] = zz.w;
    t[i][0] = tt.x, t[i][1] = tt.y, t[i][2] = tt.z, t[i][3] = tt.w;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) mx = fmaxf(mx, z[i][e]);
  mx = rows_reduce<float, NTR / 64>(mx, redf, true);
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      z[i][e] = __expf(z[i][e] - mx);  // padding: exp(-inf) = 0 (hardware exp2: ~2 ulp)
      se += z[i][e];
    }
  se = rows_reduce<float, NTR / 64>(se, redf, false);
  const float inv = 1.f / se;
  // per-thread partials in fp32 (<= 4 NV terms each; fp64 across threads), log of the ratio as
  // a difference of hardware logs: the f64 adds and the IEEE divide + log per element made this
  // kernel VALU-bound at twice its HBM time
  float klf = 0.f, Sf32 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if ((int)threadIdx.x + i * NTR >= V4) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float p = z[i][e] * inv;
      const float tc = fminf(fmaxf(t[i][e], 1e-7f), 1.f);
      const float q = fminf(fmaxf(p, 1e-7f), 1.f);
      klf += tc * (__logf(tc) - __logf(q));
      if (p >= 1e-7f) Sf32 += tc;
      z[i][e] = p;
      t[i][e] = p >= 1e-7f ? -tc : 0.f;
    }
  }
  double kl = (double)klf, S = (double)Sf32;
  rows_reduce2<NTR / 64>(kl, S, redd);
  const float Sf = (float)S;
  // dZ and, with zq, its MX-FP8 row image (K = V; columns [V, ldzq) zero codes) as cc_quant_mx8
  // makes it from the bf16 dZ: the 8 lanes of a 32-column block share its scale.  One pass: the
  // element values are computed once for both
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = threadIdx.x + i * NTR;
    if (!zq && j >= V4) break;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = scale * (t[i][e] + z[i][e] * Sf);
    if (j < V4) {
      if constexpr (sizeof(T) == 2) {
        uint2 pk = make_uint2((uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16),
                              (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16));
        reinterpret_cast<uint2 *>(dZ + (int64_t)b * V)[j] = pk;
      } else {
        reinterpret_cast<float4 *>(dZ + (int64_t)b * V)[j] = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    if (zq) {
      float v[4], amax = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = j < V4 ? bf2f(f2bf(o[e])) : 0.f;
        amax = fmaxf(amax, fabsf(v[e]));
      }
      amax = fmaxf(amax, __shfl_xor(amax, 1));
      amax = fmaxf(amax, __shfl_xor(amax, 2));
      amax = fmaxf(amax, __shfl_xor(amax, 4));
      const int ex = cc_mx8::block_exp(amax);
      int word = 0;
      word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[0], -ex), ldexpf(v[1], -ex), word, false);
      word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[2], -ex), ldexpf(v[3], -ex), word, true);
      if (j < ldzq / 4) {
        reinterpret_cast<uint32_t *>(zq + (int64_t)b * ldzq)[j] = (uint32_t)word;
        if ((j & 7) == 0) zqs[(int64_t)b * (ldzq / 32) + j / 8] = (uint8_t)(ex + 127);
      }
    }
  }
  if (threadIdx.x == 0) kl_part[b] = kl;
}

// TF ResourceApplyAdam: alpha = lr sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
// p -= m*alpha/(sqrt(v)+eps).  t = state[0] + 1.

__global__ __launch_bounds__(NT) void adam_kernel(cc_adam::Args a, const int64_t *__restrict__ state) {
  cc_adam::range(a, state[0], blockIdx.x, gridDim.x);
}

// Adam fused with the transposed bf16 operand copies (Wo^T, tower W^T): the flat blocks update
// every element outside the regions; each tile block updates one 64x64 tile of a region's
// [rows][cols] matrix, writes p/m/v and the bf16 shadow row-major, and the bf16 values
// transposed to dst [cols][rows] through LDS (both stores coalesced).  Replaces cc_adam_dense
// followed by cc_transpose / cc_tower_transpose (one launch, no re-read of the shadow).
constexpr int MAXR = 12;
struct TRegs {
  int n;
  int64_t off[MAXR], size[MAXR];
  int rows[MAXR], cols[MAXR], tcols[MAXR];
  int64_t tile0[MAXR + 1];
  bf16_t *dst[MAXR];
};

__device__ __forceinline__ void adam_tile(float *__restrict__ p, float *__restrict__ m,
                                          float *__restrict__ v, const float *__restrict__ g,
                                          bf16_t *__restrict__ shadow, const TRegs &tr,
                                          int flat_blocks, float alpha, float omb1, float omb2,
                                          float eps);

__global__ __launch_bounds__(NT) void adam_fused_kernel(float *__restrict__ p, float *__restrict__ m,
                                                        float *__restrict__ v,
                                                        const float *__restrict__ g,
                                                        bf16_t *__restrict__ shadow, int64_t n4v,
                                                        int64_t *state, float lr,
                                                        float b1, float b2, float eps, TRegs tr,
                                                        int flat_blocks, int64_t advance_bpe) {
  const float t = (float)(state[0] + 1);
  const float b1p = powf(b1, t), b2p = powf(b2, t);
  const float alpha = lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float omb1 = 1.f - b1, omb2 = 1.f - b2;
  if ((int)blockIdx.x < flat_blocks) {
    const int64_t stride = (int64_t)flat_blocks * blockDim.x;
    for (int64_t vi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; vi < n4v; vi += stride) {
      int64_t e = vi << 2;  // virtual (regions removed) -> physical element index
      for (int k = 0; k < tr.n; ++k)
        if (e >= tr.off[k]) e += tr.size[k];
      const int64_t i = e >> 2;
      float4 pp = reinterpret_cast<float4 *>(p)[i];
      float4 mm = reinterpret_cast<float4 *>(m)[i];
      float4 vv = reinterpret_cast<float4 *>(v)[i];
      const float4 gg = reinterpret_cast<const float4 *>(g)[i];
      float *pe = &pp.x, *me = &mm.x, *ve = &vv.x;
      const float *ge = &gg.x;
#pragma unroll
      for (int q = 0; q < 4; ++q) cc_adam::elem(pe[q], me[q], ve[q], ge[q], alpha, omb1, omb2, eps);
      reinterpret_cast<float4 *>(p)[i] = pp;
      reinterpret_cast<float4 *>(m)[i] = mm;
      reinterpret_cast<float4 *>(v)[i] = vv;
      ushort4 sh;
      sh.x = f2bf(pp.x);
      sh.y = f2bf(pp.y);
      sh.z = f2bf(pp.z);
      sh.w = f2bf(pp.w);
      reinterpret_cast<ushort4 *>(shadow)[i] = sh;
    }
  } else {
    adam_tile(p, m, v, g, shadow, tr, flat_blocks, alpha, omb1, omb2, eps);
  }
  if (advance_bpe > 0) {  // the last block to finish advances {step, batch, epoch}
    __syncthreads();
    if (threadIdx.x == 0) {  // no data hand-off: the ticket alone orders the counter update
      const unsigned long long tk = atomicAdd(reinterpret_cast<unsigned long long *>(state + 3), 1ull);
      if (tk == (unsigned long long)gridDim.x - 1) {  // every block has read state[0]
        state[0] += 1;
        state[1] += 1;
        if (state[1] >= advance_bpe) {
          state[1] = 0;
          state[2] += 1;
        }
        state[3] = 0;
      }
    }
  }
}

__device__ __forceinline__ void adam_tile(float *__restrict__ p, float *__restrict__ m,
                                          float *__restrict__ v, const float *__restrict__ g,
                                          bf16_t *__restrict__ shadow, const TRegs &tr,
                                          int flat_blocks, float alpha, float omb1, float omb2,
                                          float eps) {
  __shared__ bf16_t T[64][66];
  const int64_t tb = (int64_t)blockIdx.x - flat_blocks;
  int k = 0;
  while (k + 1 < tr.n && tb >= tr.tile0[k + 1]) ++k;
  const int64_t tl = tb - tr.tile0[k];
  const int rows = tr.rows[k], cols = tr.cols[k];
  const int r0 = (int)(tl / tr.tcols[k]) * 64, c0 = (int)(tl % tr.tcols[k]) * 64;
  const int64_t base = tr.off[k];
  // 64 x 64 tile as 1024 float4 (16 per row): every load of the thread is issued before any
  // math (a load -> math -> store chain per element would expose the memory latency 16 times)
  constexpr int Q = 64 * 16 / NT;
  float4 P4[Q], M4[Q], V4[Q], G4[Q];
  bool ok[Q];
#pragma unroll
  for (int qq = 0; qq < Q; ++qq) {
    const int q = threadIdx.x + NT * qq, rr = q >> 4, c = c0 + (q & 15) * 4, r = r0 + rr;
    ok[qq] = r < rows && c + 3 < cols && (cols & 3) == 0;
    if (ok[qq]) {
      const int64_t i4 = (base + (int64_t)r * cols + c) >> 2;
      P4[qq] = reinterpret_cast<const float4 *>(p)[i4];
      M4[qq] = reinterpret_cast<const float4 *>(m)[i4];
      V4[qq] = reinterpret_cast<const float4 *>(v)[i4];
      G4[qq] = reinterpret_cast<const float4 *>(g)[i4];
    }
  }
#pragma unroll
  for (int qq = 0; qq < Q; ++qq) {
    const int q = threadIdx.x + NT * qq, rr = q >> 4, cl = (q & 15) * 4, c = c0 + cl, r = r0 + rr;
    if (ok[qq]) {
      float *pe = &P4[qq].x, *me = &M4[qq].x, *ve = &V4[qq].x;
      const float *ge = &G4[qq].x;
#pragma unroll
      for (int e = 0; e < 4; ++e) cc_adam::elem(pe[e], me[e], ve[e], ge[e], alpha, omb1, omb2, eps);
      const int64_t i4 = (base + (int64_t)r * cols + c) >> 2;
      reinterpret_cast<float4 *>(p)[i4] = P4[qq];
      reinterpret_cast<float4 *>(m)[i4] = M4[qq];
      reinterpret_cast<float4 *>(v)[i4] = V4[qq];
      ushort4 sh;
      sh.x = f2bf(pe[0]);
      sh.y = f2bf(pe[1]);
      sh.z = f2bf(pe[2]);
      sh.w = f2bf(pe[3]);
      reinterpret_cast<ushort4 *>(shadow)[i4] = sh;
      T[rr][cl] = sh.x;
      T[rr][cl + 1] = sh.y;
      T[rr][cl + 2] = sh.z;
      T[rr][cl + 3] = sh.w;
    } else if (r < rows) {  // ragged edge (or cols % 4 != 0): element by element
      for (int e = 0; e < 4 && c + e < cols; ++e) {
        const int64_t i = base + (int64_t)r * cols + c + e;
        float pp = p[i], mm = m[i], vv = v[i];
        cc_adam::elem(pp, mm, vv, g[i], alpha, omb1, omb2, eps);
        p[i] = pp;
        m[i] = mm;
        v[i] = vv;
        const bf16_t b = f2bf(pp);
        shadow[i] = b;
        T[rr][cl + e] = b;
      }
    }
  }
  __syncthreads();
  bf16_t *dst = tr.dst[k];
  for (int e = threadIdx.x; e < 64 * 64; e += NT) {  // dst row c0 + e/64: 64 consecutive rows
    const int cc = e >> 6, rr = e & 63;
    const int c = c0 + cc, r = r0 + rr;
    if (r < rows && c < cols) dst[(int64_t)c * rows + r] = T[rr][cc];
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
                                       const float *y_reg, const int32_t *reg_idx, float scale,
                                       void *dZ, double *kl_partials, void *stream) {
  CC_REQUIRE(Z2 && y_reg && reg_idx && dZ && kl_partials, "cc_dec_softmax_kl_fused: null pointer");
  if (B == 0) return CC_OK;
  const bool aligned = (V % 4 == 0) && ((uintptr_t)Z2 % 16 == 0) && ((uintptr_t)y_reg % 16 == 0) &&
                       ((uintptr_t)dZ % 16 == 0);
  const int nv = (int)cdiv(V, 4 * NTR);
  if (aligned && nv <= 8) {  // register-resident rows
    const hipStream_t s = as_stream(stream);
#define KL_ROWS(NVV)                                                                            \
  if (nv <= NVV) {                                                                              \
    if (dtype == CC_BF16)                                                                       \
      hipLaunchKernelGGL((softmax_kl_rows_kernel<bf16_t, NVV>), dim3(B), dim3(NTR), 0, s, Z2, V, \
                         y_reg, reg_idx, scale, (bf16_t *)dZ, kl_partials);                     \
    else                                                                                        \
      hipLaunchKernelGGL((softmax_kl_rows_kernel<float, NVV>), dim3(B), dim3(NTR), 0, s, Z2, V,  \
                         y_reg, reg_idx, scale, (float *)dZ, kl_partials);                      \
    CC_LAUNCH_CHECK("softmax_kl_rows_kernel");                                                  \
    return CC_OK;                                                                               \
  }
    KL_ROWS(1)
    KL_ROWS(2)
    KL_ROWS(4)
    KL_ROWS(6)
    KL_ROWS(8)
#undef KL_ROWS
  }
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
  const int64_t blocks = std::min<int64_t>(cdiv(cdiv(n, 4), NT), 1 << 30);  // one float4 per thread
  const cc_adam::Args a{p, m, v, g, (bf16_t *)shadow, n, lr, beta1, beta2, eps};
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(NT), 0, as_stream(stream), a, state);
  CC_LAUNCH_CHECK("adam_kernel");
  return CC_OK;
}

extern "C" int cc_adam_dense_t(float *p, float *m, float *v, const float *g, uint16_t *shadow,
                               int64_t n, int64_t *state, float lr, float beta1,
                               float beta2, float eps, const cc_adam_tregion *regions,
                               int32_t nregions, int64_t advance_bpe, void *stream) {
  CC_REQUIRE(p && m && v && g && state && shadow, "cc_adam_dense_t: null pointer");
  CC_REQUIRE(((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g) % 16 == 0,
             "cc_adam_dense_t: buffers must be 16-byte aligned");
  CC_REQUIRE((uintptr_t)shadow % 8 == 0, "cc_adam_dense_t: shadow must be 8-byte aligned");
  CC_REQUIRE(n % 4 == 0, "cc_adam_dense_t: n must be a multiple of 4");
  CC_REQUIRE(nregions >= 0 && nregions <= MAXR && (nregions == 0 || regions),
             "cc_adam_dense_t: 0..12 regions");
  TRegs tr{};
  tr.n = nregions;
  int64_t covered = 0, prev_end = 0, tiles = 0;
  for (int k = 0; k < nregions; ++k) {
    const cc_adam_tregion &r = regions[k];
    const int64_t size = (int64_t)r.rows * r.cols;
    CC_REQUIRE(r.dst && r.rows > 0 && r.cols > 0, "cc_adam_dense_t: empty region");
    CC_REQUIRE(r.off >= prev_end && r.off + size <= n, "cc_adam_dense_t: regions must be sorted, disjoint, in range");
    CC_REQUIRE(r.off % 4 == 0 && size % 4 == 0, "cc_adam_dense_t: regions must be 4-element aligned");
    tr.off[k] = r.off;
    tr.size[k] = size;
    tr.rows[k] = r.rows;
    tr.cols[k] = r.cols;
    tr.tcols[k] = (int)cdiv(r.cols, 64);
    tr.dst[k] = (bf16_t *)r.dst;
    tr.tile0[k] = tiles;
    tiles += cdiv(r.rows, 64) * tr.tcols[k];
    covered += size;
    prev_end = r.off + size;
  }
  tr.tile0[nregions] = tiles;
  const int64_t n4v = (n - covered) / 4;
  const int flat_blocks = n4v > 0 ? (int)std::min<int64_t>(cdiv(n4v, NT), 256 * 8) : 0;
  const int64_t blocks = flat_blocks + tiles;
  if (blocks == 0) return CC_OK;
  hipLaunchKernelGGL(adam_fused_kernel, dim3((unsigned)blocks), dim3(NT), 0, as_stream(stream), p,
                     m, v, g, (bf16_t *)shadow, n4v, state, lr, beta1, beta2, eps, tr, flat_blocks,
                     advance_bpe);
  CC_LAUNCH_CHECK("adam_fused_kernel");
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

// cc_dec_softmax_kl_fused (bf16 dZ) that also writes the MX-FP8 row image of dZ (zq [B][ldzq] codes,
// zqs [B][ldzq/32] scales; bit-exact with cc_quant_mx8 of the bf16 dZ): config 5's regulariser
// branch without the separate row quantiser launch
extern "C" int cc_dec_softmax_kl_q(const float *Z2, int32_t B, int32_t V, const float *y_reg,
                                   const int32_t *reg_idx, float scale, void *dZ, double *kl_partials,
                                   uint8_t *zq, int32_t ldzq, uint8_t *zqs, void *stream) {
  CC_REQUIRE(Z2 && y_reg && reg_idx && dZ && kl_partials && zq && zqs, "cc_dec_softmax_kl_q: null pointer");
  CC_REQUIRE(ldzq % 128 == 0 && ldzq >= V && (uintptr_t)zq % 4 == 0, "cc_dec_softmax_kl_q: ldzq % 128, >= V");
  CC_REQUIRE((V % 4 == 0) && ((uintptr_t)Z2 % 16 == 0) && ((uintptr_t)y_reg % 16 == 0) && ((uintptr_t)dZ % 16 == 0),
             "cc_dec_softmax_kl_q: V % 4 == 0, 16-B aligned rows");
  if (B == 0) return CC_OK;
  const int nv = (int)cdiv(ldzq, 4 * NTR);
  CC_REQUIRE(nv <= 8, "cc_dec_softmax_kl_q: ldzq <= 32768");
  const hipStream_t s = as_stream(stream);
#define KL_ROWS_Q(NVV)                                                                              \
  if (nv <= NVV) {                                                                                  \
    hipLaunchKernelGGL((softmax_kl_rows_kernel<bf16_t, NVV>), dim3(B), dim3(NTR), 0, s, Z2, V, y_reg, \
                       reg_idx, scale, (bf16_t *)dZ, kl_partials, zq, ldzq, zqs);                   \
    CC_LAUNCH_CHECK("softmax_kl_rows_kernel<q>");                                                   \
    return CC_OK;                                                                                   \
  }
  KL_ROWS_Q(1)
  KL_ROWS_Q(2)
  KL_ROWS_Q(4)
  KL_ROWS_Q(6)
  KL_ROWS_Q(8)
#undef KL_ROWS_Q
  return CC_OK;
}
