// Shared device/host helpers for libccrec_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "ccrec.h"

typedef uint16_t bf16_t;  // bfloat16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

#define CC_WAVE 64

// The hardware deals a launch's workgroups to the 8 XCDs round robin (block b on XCD b % 8).  This
// bijection gives each XCD a contiguous run of ids, so workgroups whose data share 128-B lines
// (neighbouring column slices) fetch them into one L2 instead of several.
__device__ __forceinline__ int cc_xcd_run(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8, slot = b / 8;
  return x < r ? x * (q + 1) + slot : r * (q + 1) + (x - r) * q + slot;
}
// CCREC_XCD_SLICES (build knob for the A/B, default on): the fused output-layer kernels (D1's
// dec_bce_dw, D2's kl_stats / kl_main) take their 96-column slice from cc_xcd_run instead of
// blockIdx.x
#ifndef CCREC_XCD_SLICES
#define CCREC_XCD_SLICES 1
#endif
__device__ __forceinline__ int cc_slice_of_block(int b, int nb) { return CCREC_XCD_SLICES ? cc_xcd_run(b, nb) : b; }

// ------------------------------------------------------------------ error plumbing (host)
namespace cc {
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
}  // namespace cc

#define CC_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t _e = (call);                                                            \
    if (_e != hipSuccess)                                                              \
      return cc::fail(CC_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e));  \
  } while (0)

#define CC_LAUNCH_CHECK(name)                                                             \
  do {                                                                                    \
    hipError_t _e = hipGetLastError();                                                    \
    if (_e != hipSuccess)                                                                 \
      return cc::fail(CC_ERR_HIP, std::string(name) + " launch: " + hipGetErrorString(_e)); \
  } while (0)

#define CC_REQUIRE(cond, msg) \
  do {                        \
    if (!(cond)) return cc::fail(CC_ERR_ARG, msg); \
  } while (0)

static inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------ bf16 helpers (device)
__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
// Round-to-nearest-even (inputs are finite); identical to oracle/model_ref.py::bf16_round.
__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

template <typename T> struct DT;
template <> struct DT<float> {
  static __device__ __forceinline__ float ld(const float *p) { return *p; }
  static __device__ __forceinline__ void st(float *p, float v) { *p = v; }
  static constexpr int code = CC_F32;
};
template <> struct DT<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t *p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t *p, float v) { *p = f2bf(v); }
  static constexpr int code = CC_BF16;
};

__host__ __device__ static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------ Philox4x32-10 (device)
struct u32x4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return {c0, c1, c2, c3};
}
__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
  const uint64_t a = ((uint64_t)hi << 32) | lo;
  return (double)(a >> 11) * 0x1.0p-53;
}
__device__ __forceinline__ double u53_open0(uint32_t hi, uint32_t lo) {
  const uint64_t a = ((uint64_t)hi << 32) | lo;
  return (double)((a >> 11) + 1) * 0x1.0p-53;
}
__device__ __forceinline__ uint32_t mulhi_bound(uint32_t x, uint32_t n) {
  return (uint32_t)(((uint64_t)x * (uint64_t)n) >> 32);
}

// L2 warm-up for the NEXT launch, called at the end of a kernel: workgroups are dispatched
// round-robin over the 8 XCDs (block b -> XCD b % 8), so the blocks of one XCD together read one
// dword per 128-B line of [p, p + bytes) and the next kernel finds those lines in every XCD's L2.
__device__ __forceinline__ void l2_warm(const void *p, int64_t bytes, int block, int nblocks) {
  if (!p || bytes <= 0 || nblocks < 8) return;
  const int per = nblocks / 8;
  if (block >= per * 8) return;
  const int part = block / 8;
  const int64_t lines = (bytes + 127) / 128, chunk = (lines + per - 1) / per;
  const int64_t l0 = (int64_t)part * chunk, l1 = l0 + chunk < lines ? l0 + chunk : lines;
  uint32_t acc = 0u;
  for (int64_t l = l0 + threadIdx.x; l < l1; l += blockDim.x) acc += reinterpret_cast<const uint32_t *>(p)[l * 32];
  asm volatile("" ::"v"(acc));
}
