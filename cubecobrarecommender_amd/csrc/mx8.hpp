// MX-FP8 block rule shared by the quantiser (mx8.hip) and the producers that emit MX-FP8 operand
// images themselves (tower.hip: D3 for config 5).  One E8M0 scale per 32 elements along the GEMM's
// K axis, restated in oracle/mx8_ref.py (bit-exact):
//   e = min{e : amax <= 448 * 2^e} (= x - 9 + (m > 0.875) for amax = m 2^x), e in [-127, 127];
//   code = OCP e4m3fn round-to-nearest-even of v * 2^-e (v_cvt_pk_fp8_f32); never saturates.
#pragma once
#include "common.hpp"

namespace cc_mx8 {

__device__ __forceinline__ int block_exp(float amax) {
  if (!(amax > 0.f)) return 0;
  int x;
  const float m = frexpf(amax, &x);
  int e = x - 9 + (m > 0.875f ? 1 : 0);
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

// 32 values -> 32 e4m3 codes (little-endian bytes in w[8]) at scale 2^-e
__device__ __forceinline__ void encode32(const float *v, int e, uint32_t *w) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    int word = 0;
    word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * q], -e), ldexpf(v[4 * q + 1], -e), word, false);
    word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * q + 2], -e), ldexpf(v[4 * q + 3], -e), word, true);
    w[q] = (uint32_t)word;
  }
}

}  // namespace cc_mx8
