// MX-FP8 quantisation of GEMM operands (config 5, SURVEY §8(d): the decoder output layer and the
// regulariser GEMM of model.py:64,94,98 on v_mfma_scale_f32_32x32x64_f8f6f4).  One E8M0 scale per
// 32 elements along the GEMM's K axis; the rule is restated in oracle/mx8_ref.py (bit-exact):
//   e = min{e : amax <= 448 * 2^e} (= x - 9 + (m > 0.875) for amax = m 2^x), e in [-127, 127];
//   code = OCP e4m3fn round-to-nearest-even of v * 2^-e (v_cvt_pk_fp8_f32); never saturates.
// Row blocks: one lane per 32-element block (two 16-B stores per lane).  Transposed blocks: a
// workgroup stages a [32 rows][256 cols] tile in LDS and each lane emits one output row's block.
#include "common.hpp"
#include "mx8.hpp"

namespace {

template <typename T>
__device__ __forceinline__ float ldf(const T *p, int64_t i) { return DT<T>::ld(p + i); }

using cc_mx8::block_exp;
using cc_mx8::encode32;

// grid (ceil(nb / 64), rows), block 64: lane -> block j of row r; with rowsum (gridDim.x == 1) the
// wave also sums the row (per-lane ascending partials, then a fixed xor tree: deterministic).
template <typename T>
__global__ __launch_bounds__(64) void quant_rows_kernel(const T *__restrict__ src, int cols, int ld_src,
                                                        uint8_t *__restrict__ dst, int ld_dst,
                                                        uint8_t *__restrict__ scales,
                                                        float *__restrict__ rowsum) {
  const int r = blockIdx.y, nb = ld_dst / 32;
  const T *row = src + (int64_t)r * ld_src;
  float part = 0.f;
  for (int j = blockIdx.x * 64 + threadIdx.x; j < nb; j += gridDim.x * 64) {
    float v[32];
    const int c0 = 32 * j;
    if (c0 + 32 <= cols && sizeof(T) == 2 && (ld_src % 8) == 0 && ((uintptr_t)src % 16) == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 u = *reinterpret_cast<const uint4 *>(row + c0 + 8 * q);
        const uint32_t uw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[8 * q + 2 * e] = __uint_as_float(uw[e] << 16);
          v[8 * q + 2 * e + 1] = __uint_as_float(uw[e] & 0xFFFF0000u);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 32; ++e) v[e] = c0 + e < cols ? ldf(row, c0 + e) : 0.f;
    }
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      amax = fmaxf(amax, fabsf(v[e]));
      part += v[e];
    }
    const int ex = block_exp(amax);
    uint32_t w[8];
    encode32(v, ex, w);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst + (int64_t)r * ld_dst + c0);
    d4[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d4[1] = make_uint4(w[4], w[5], w[6], w[7]);
    scales[(int64_t)r * nb + j] = (uint8_t)(ex + 127);
  }
  if (rowsum) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) part += __shfl_xor(part, off);
    if (threadIdx.x == 0) rowsum[r] = part;
  }
}

// Transposed: dst[c][r] = q(src[r][c]); K axis = r.  grid (ceil(cols / 64), ld_dst / 128), block
// 256: tile rows [128 by, +128), cols [64 bx, +64) (a whole 128-B line of every bf16 source row);
// thread (rb = tid / 64, c = tid % 64) emits dst row (64 bx + c)'s block 4 by + rb, so the four
// waves of a block write one whole 128-B line of each of its 64 dst rows.
constexpr int QT_C = 64, QT_R = 128;
// ROWS: the same tile also yields the row image (K = cols): 128 rows x 2 blocks of 32 columns, one
// block per thread, from the staged tile — both images of a weight from one read of it
template <typename T, bool ROWS = false>
__global__ __launch_bounds__(256) void quant_t_kernel(const T *__restrict__ src, int rows, int cols,
                                                      int ld_src, uint8_t *__restrict__ dst, int ld_dst,
                                                      uint8_t *__restrict__ scales, uint8_t *__restrict__ dst_r = nullptr,
                                                      int ld_r = 0, uint8_t *__restrict__ scales_r = nullptr) {
  __shared__ float tile[QT_R][QT_C + 1];
  const int c0 = blockIdx.x * QT_C, r0 = blockIdx.y * QT_R;
  if (sizeof(T) == 2 && c0 + QT_C <= cols && (ld_src % 8) == 0 && ((uintptr_t)src % 16) == 0) {
    // full-width bf16 tile: 16-B loads, all of a thread's issued before any LDS store
    constexpr int NV = QT_R * QT_C / 8 / 256;  // 16-B vectors per thread
    uint4 u[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int i = threadIdx.x + q * 256, rr = i / (QT_C / 8), cc = (i % (QT_C / 8)) * 8;
      const int gr = min(r0 + rr, rows - 1);
      u[q] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint16_t *>(src) + (int64_t)gr * ld_src + c0 + cc);
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int i = threadIdx.x + q * 256, rr = i / (QT_C / 8), cc = (i % (QT_C / 8)) * 8;
      const bool ok = r0 + rr < rows;
      const uint32_t uw[4] = {u[q].x, u[q].y, u[q].z, u[q].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        tile[rr][cc + 2 * e] = ok ? __uint_as_float(uw[e] << 16) : 0.f;
        tile[rr][cc + 2 * e + 1] = ok ? __uint_as_float(uw[e] & 0xFFFF0000u) : 0.f;
      }
    }
  } else {
    for (int i = threadIdx.x; i < QT_R * QT_C; i += 256) {
      const int rr = i / QT_C, cc = i % QT_C;
      const int gr = r0 + rr, gc = c0 + cc;
      tile[rr][cc] = gr < rows && gc < cols ? ldf(src, (int64_t)gr * ld_src + gc) : 0.f;
    }
  }
  __syncthreads();
  const int cl = threadIdx.x % QT_C, rb = threadIdx.x / QT_C;
  const int c = c0 + cl;
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int e = 0; e < 32; ++e) {
    v[e] = tile[32 * rb + e][cl];
    amax = fmaxf(amax, fabsf(v[e]));
  }
  const int ex = block_exp(amax);
  uint32_t w[8];
  encode32(v, ex, w);
  if (c < cols) scales[(int64_t)c * (ld_dst / 32) + 4 * blockIdx.y + rb] = (uint8_t)(ex + 127);
  if constexpr (ROWS) {  // row blocks (K = cols): thread -> row t / 2, columns 32 (t & 1) .. + 32
    const int rr = threadIdx.x >> 1, b = threadIdx.x & 1;
    float u[32];
    float um = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      u[e] = tile[rr][32 * b + e];   // zero past cols (and past rows)
      um = fmaxf(um, fabsf(u[e]));
    }
    const int eu = block_exp(um);
    uint32_t wu[8];
    encode32(u, eu, wu);
    if (r0 + rr < rows) {
      uint4 *d4 = reinterpret_cast<uint4 *>(dst_r + (int64_t)(r0 + rr) * ld_r + c0 + 32 * b);
      d4[0] = make_uint4(wu[0], wu[1], wu[2], wu[3]);
      d4[1] = make_uint4(wu[4], wu[5], wu[6], wu[7]);
      scales_r[(int64_t)(r0 + rr) * (ld_r / 32) + c0 / 32 + b] = (uint8_t)(eu + 127);
    }
  }
  // re-lay the codes through LDS so each store instruction writes whole 128-B lines (8 lanes per dst
  // row) instead of 64 scattered 16-B pieces; rows padded to 9 x 16 B against bank conflicts
  __syncthreads();
  uint4 *ot = reinterpret_cast<uint4 *>(&tile[0][0]);
  ot[cl * 9 + 2 * rb] = make_uint4(w[0], w[1], w[2], w[3]);
  ot[cl * 9 + 2 * rb + 1] = make_uint4(w[4], w[5], w[6], w[7]);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = threadIdx.x + 256 * q, rr = i / 8, sg = i % 8;
    if (c0 + rr < cols)
      *reinterpret_cast<uint4 *>(dst + (int64_t)(c0 + rr) * ld_dst + r0 + 16 * sg) = ot[rr * 9 + sg];
  }
}

}  // namespace

extern "C" int cc_quant_mx8(int32_t dtype, const void *src, int32_t rows, int32_t cols, int32_t ld_src,
                            int32_t transpose, uint8_t *dst, int32_t ld_dst, uint8_t *scales,
                            float *rowsum, void *stream) {
  CC_REQUIRE(src && dst && scales, "cc_quant_mx8: null pointer");
  CC_REQUIRE(dtype == CC_BF16 || dtype == CC_F32, "cc_quant_mx8: dtype");
  CC_REQUIRE(rows >= 0 && cols >= 0 && ld_src >= cols, "cc_quant_mx8: shape");
  CC_REQUIRE(ld_dst % 128 == 0 && (uintptr_t)dst % 16 == 0, "cc_quant_mx8: ld_dst % 128, dst 16-B aligned");
  if (rows == 0 || cols == 0) return CC_OK;
  hipStream_t s = as_stream(stream);
  if (!transpose) {
    CC_REQUIRE(ld_dst >= cols, "cc_quant_mx8: ld_dst < cols");
    const int nb = ld_dst / 32;
    CC_REQUIRE(!rowsum || nb <= 64, "cc_quant_mx8: rowsum needs ld_dst <= 2048");
    const dim3 grid(rowsum ? 1u : (unsigned)cdiv(nb, 64), (unsigned)rows);
    if (dtype == CC_BF16)
      hipLaunchKernelGGL(quant_rows_kernel<bf16_t>, grid, dim3(64), 0, s, (const bf16_t *)src, cols, ld_src,
                         dst, ld_dst, scales, rowsum);
    else
      hipLaunchKernelGGL(quant_rows_kernel<float>, grid, dim3(64), 0, s, (const float *)src, cols, ld_src,
                         dst, ld_dst, scales, rowsum);
    CC_LAUNCH_CHECK("quant_rows_kernel");
    return CC_OK;
  }
  CC_REQUIRE(!rowsum, "cc_quant_mx8: rowsum only without transpose");
  CC_REQUIRE(ld_dst >= rows, "cc_quant_mx8: ld_dst < rows");
  const dim3 grid((unsigned)cdiv(cols, QT_C), (unsigned)(ld_dst / QT_R));
  if (dtype == CC_BF16)
    hipLaunchKernelGGL(quant_t_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t *)src, rows, cols, ld_src,
                       dst, ld_dst, scales);
  else
    hipLaunchKernelGGL(quant_t_kernel<float>, grid, dim3(256), 0, s, (const float *)src, rows, cols, ld_src,
                       dst, ld_dst, scales);
  CC_LAUNCH_CHECK("quant_t_kernel");
  return CC_OK;
}

// Both MX-FP8 images of one weight from a single read of it (config 5's decoder output kernel Wo
// [d][V] after every Adam step): the transposed image dst_t [cols][ld_t] (K = rows, the forward
// product's B operand) and the row image dst_r [rows][ld_r] (K = cols, the dX product's B operand,
// columns [cols, ld_r) zero codes) — each bit-exact with cc_quant_mx8 of the same source.
extern "C" int cc_quant_mx8_both(int32_t dtype, const void *src, int32_t rows, int32_t cols, int32_t ld_src,
                                 uint8_t *dst_t, int32_t ld_t, uint8_t *scales_t, uint8_t *dst_r, int32_t ld_r,
                                 uint8_t *scales_r, void *stream) {
  CC_REQUIRE(src && dst_t && scales_t && dst_r && scales_r, "cc_quant_mx8_both: null pointer");
  CC_REQUIRE(dtype == CC_BF16 || dtype == CC_F32, "cc_quant_mx8_both: dtype");
  CC_REQUIRE(rows >= 0 && cols >= 0 && ld_src >= cols, "cc_quant_mx8_both: shape");
  CC_REQUIRE(ld_t % 128 == 0 && ld_t >= rows && ld_r % 128 == 0 && ld_r >= cols &&
                 (((uintptr_t)dst_t | (uintptr_t)dst_r) & 15) == 0,
             "cc_quant_mx8_both: ld_t, ld_r multiples of 128 covering rows / cols, images 16-B aligned");
  if (rows == 0 || cols == 0) return CC_OK;
  const dim3 grid((unsigned)cdiv(ld_r, QT_C), (unsigned)(ld_t / QT_R));
  hipStream_t s = as_stream(stream);
  if (dtype == CC_BF16)
    hipLaunchKernelGGL((quant_t_kernel<bf16_t, true>), grid, dim3(256), 0, s, (const bf16_t *)src, rows, cols, ld_src,
                       dst_t, ld_t, scales_t, dst_r, ld_r, scales_r);
  else
    hipLaunchKernelGGL((quant_t_kernel<float, true>), grid, dim3(256), 0, s, (const float *)src, rows, cols, ld_src,
                       dst_t, ld_t, scales_t, dst_r, ld_r, scales_r);
  CC_LAUNCH_CHECK("quant_t_kernel<rows>");
  return CC_OK;
}
