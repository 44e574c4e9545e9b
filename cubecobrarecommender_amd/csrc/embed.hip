// E1 — the sparse-binary-cube encoder input layer (model.py:27,36: Dense(d, relu) on a 0/1
// cube vector), as an embedding-row gather instead of a dense [R,V]x[V,d] GEMM, and its
// backward (the dense MatMul gradient of that layer), as a row-owner reduction that needs
// no float atomics.
//
// Forward  cc_embed_gather_fwd : one wave per cube row; lane l owns d/64 consecutive columns;
//   the row's sorted card list is walked in order with EPL-wide vector loads of W1 rows
//   (bf16 shadow: 8..16 B per lane; fp32: 16..32 B) — each W1 row is one coalesced wave access.
// Backward cc_embed_scatter_bwd: one wave per W1 row r; the transposed bitmask xt_bits[r] lists
//   the batch rows containing card r; their dPre rows (L2-resident, [R, d] fp32) are summed in
//   ascending row order — deterministic, and dense over every row (rows absent from the batch
//   get an exact zero gradient, as TF's dense MatMul gradient gives).
#include "common.hpp"

namespace {

template <typename T, int EPL>
__global__ __launch_bounds__(256) void gather_kernel(const T *__restrict__ table,
                                                     const float *__restrict__ bias, int d, int R,
                                                     const int32_t *__restrict__ x_cnt,
                                                     const int32_t *__restrict__ x_idx, int x_cap,
                                                     T *__restrict__ out) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= R) return;
  const int c0 = lane * EPL;
  float acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
  const int n = x_cnt[wave];
  const int32_t *__restrict__ lst = x_idx + (int64_t)wave * x_cap;
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    const int j0 = lst[i], j1 = lst[i + 1], j2 = lst[i + 2], j3 = lst[i + 3];
    const T *r0 = table + (int64_t)j0 * d + c0;
    const T *r1 = table + (int64_t)j1 * d + c0;
    const T *r2 = table + (int64_t)j2 * d + c0;
    const T *r3 = table + (int64_t)j3 * d + c0;
    float v0[EPL], v1[EPL], v2[EPL], v3[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      v0[e] = DT<T>::ld(r0 + e);
      v1[e] = DT<T>::ld(r1 + e);
      v2[e] = DT<T>::ld(r2 + e);
      v3[e] = DT<T>::ld(r3 + e);
    }
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[e] = (((acc[e] + v0[e]) + v1[e]) + v2[e]) + v3[e];
  }
  for (; i < n; ++i) {
    const T *r0 = table + (int64_t)lst[i] * d + c0;
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[e] += DT<T>::ld(r0 + e);
  }
  T *o = out + (int64_t)wave * d + c0;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const float v = acc[e] + bias[c0 + e];
    DT<T>::st(o + e, v > 0.f ? v : 0.f);
  }
}

template <int EPL>
__global__ __launch_bounds__(256) void scatter_bwd_kernel(const float *__restrict__ dpre, int V,
                                                          int d, int R,
                                                          const uint32_t *__restrict__ xt,
                                                          float *__restrict__ grad) {
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= V) return;
  const int XW = (R + 31) >> 5;
  const int c0 = lane * EPL;
  float acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
  const uint32_t *bits = xt + (int64_t)row * XW;
  for (int w = 0; w < XW; ++w) {
    uint32_t m = bits[w];
    while (m) {
      const int b = (w << 5) + __ffs(m) - 1;
      m &= m - 1;
      const float *src = dpre + (int64_t)b * d + c0;
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] += src[e];
    }
  }
  float *g = grad + (int64_t)row * d + c0;
#pragma unroll
  for (int e = 0; e < EPL; ++e) g[e] = acc[e];
}

}  // namespace

extern "C" int cc_embed_gather_fwd(int32_t dtype, const void *table, const float *bias, int32_t V,
                                   int32_t d, int32_t R, const int32_t *x_cnt,
                                   const int32_t *x_idx, int32_t x_cap, void *out, void *stream) {
  CC_REQUIRE(table && bias && x_cnt && x_idx && out, "cc_embed_gather_fwd: null pointer");
  CC_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "cc_embed_gather_fwd: d must be 64..1024, %64");
  CC_REQUIRE(V > 0 && R >= 0 && x_cap > 0, "cc_embed_gather_fwd: bad sizes");
  if (R == 0) return CC_OK;
  const dim3 grid((unsigned)cdiv((int64_t)R * 64, 256)), block(256);
  const int epl = d / 64;
  hipStream_t s = as_stream(stream);
#define GATHER_CASE(E)                                                                          \
  case E:                                                                                       \
    if (dtype == CC_BF16)                                                                       \
      hipLaunchKernelGGL((gather_kernel<bf16_t, E>), grid, block, 0, s, (const bf16_t *)table, \
                         bias, d, R, x_cnt, x_idx, x_cap, (bf16_t *)out);                      \
    else                                                                                        \
      hipLaunchKernelGGL((gather_kernel<float, E>), grid, block, 0, s, (const float *)table,   \
                         bias, d, R, x_cnt, x_idx, x_cap, (float *)out);                       \
    break;
  switch (epl) {
    GATHER_CASE(1)
    GATHER_CASE(2)
    GATHER_CASE(4)
    GATHER_CASE(8)
    GATHER_CASE(16)
    default:
      return cc::fail(CC_ERR_UNSUPPORTED, "cc_embed_gather_fwd: d/64 must be a power of two");
  }
#undef GATHER_CASE
  CC_LAUNCH_CHECK("gather_kernel");
  return CC_OK;
}

extern "C" int cc_embed_scatter_bwd(const float *dpre, int32_t V, int32_t d, int32_t R,
                                    const uint32_t *xt_bits, float *grad, void *stream) {
  CC_REQUIRE(dpre && xt_bits && grad, "cc_embed_scatter_bwd: null pointer");
  CC_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "cc_embed_scatter_bwd: d must be 64..1024, %64");
  const dim3 grid((unsigned)cdiv((int64_t)V * 64, 256)), block(256);
  hipStream_t s = as_stream(stream);
  switch (d / 64) {
    case 1: hipLaunchKernelGGL((scatter_bwd_kernel<1>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad); break;
    case 2: hipLaunchKernelGGL((scatter_bwd_kernel<2>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad); break;
    case 4: hipLaunchKernelGGL((scatter_bwd_kernel<4>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad); break;
    case 8: hipLaunchKernelGGL((scatter_bwd_kernel<8>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad); break;
    case 16: hipLaunchKernelGGL((scatter_bwd_kernel<16>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad); break;
    default: return cc::fail(CC_ERR_UNSUPPORTED, "cc_embed_scatter_bwd: d/64 must be a power of two");
  }
  CC_LAUNCH_CHECK("scatter_bwd_kernel");
  return CC_OK;
}
