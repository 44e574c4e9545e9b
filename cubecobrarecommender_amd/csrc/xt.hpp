// xt_transpose_block: the W1-gradient bitmask as the bit transpose of F's x row bitmasks, for the
// launches it rides in as extra blocks (cc_embed_gather_fwd_xt, cc_tower_fwd) and its own kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

// xt = bit transpose of the x row bitmasks: xt[j][w] bit r = x_bits[32 w + r] bit j, rows < xt_rows.
// One block per XT_TJ words of cards (32 XT_TJ cards); a wave transposes two 32 x 32 bit tiles per
// pass (lanes 0-31 tile A, 32-63 tile B) by 32 ballots, every xt word written.  The row words of
// XT_Q passes are loaded up front (unconditional clamped loads): one load latency per XT_Q passes.
#ifndef CC_XT_TJ
#define CC_XT_TJ 2
#endif
constexpr int XT_TJ = CC_XT_TJ, XT_Q = 4;
__device__ __forceinline__ void xt_transpose_block(const uint32_t *__restrict__ xb, int V,
                                                   uint32_t *__restrict__ xt, int xt_rows, int tb) {
  const int VW = (V + 31) >> 5, XW = (xt_rows + 31) >> 5;
  const int lane = threadIdx.x & 63, c = lane & 31;
  const int nw = (int)(blockDim.x >> 6), wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int npair = XW * XT_TJ;  // (row word w, card word jw) tiles of this block (even)
  for (int p0 = 2 * wv; p0 < npair; p0 += 2 * nw * XT_Q) {
    uint32_t word[XT_Q];
#pragma unroll
    for (int q = 0; q < XT_Q; ++q) {
      const int p = p0 + 2 * nw * q + (lane >> 5);
      const int w = p / XT_TJ, jw = tb * XT_TJ + p % XT_TJ, r = 32 * w + c;
      const bool ok = p < npair && r < xt_rows && jw < VW;
      const uint32_t u = xb[(int64_t)min(r, xt_rows - 1) * VW + min(jw, VW - 1)];
      word[q] = ok ? u : 0u;
    }
#pragma unroll
    for (int q = 0; q < XT_Q; ++q) {
      const int p = p0 + 2 * nw * q + (lane >> 5);
      const int w = p / XT_TJ, jw = tb * XT_TJ + p % XT_TJ;
      uint32_t out = 0u;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const uint64_t bal = __ballot((word[q] >> k) & 1u);
        const uint32_t t = lane < 32 ? (uint32_t)bal : (uint32_t)(bal >> 32);
        out = c == k ? t : out;
      }
      const int j = 32 * jw + c;
      if (p < npair && jw < VW && j < V) xt[(int64_t)j * XW + w] = out;
    }
  }
}

}  // namespace
