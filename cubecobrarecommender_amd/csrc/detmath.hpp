// Deterministic fp64 exp / log / cos(2*pi*x) for the device.  Every multiply and add is a
// separately rounded IEEE op (contraction disabled), with the same constants and operation
// order as the CPU oracle (oracle/detmath.py), so the two produce bit-identical results.
// Used by the recommend sigmoid (ranking must be bit-exact) and the F noise-level draw.
#pragma once
#include <hip/hip_runtime.h>

namespace detm {

__device__ static const double EXP_C[14] = {
    0x1.0000000000000p+0, 0x1.0000000000000p+0, 0x1.0000000000000p-1, 0x1.5555555555555p-3,
    0x1.5555555555555p-5, 0x1.1111111111111p-7, 0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-13,
    0x1.a01a01a01a01ap-16, 0x1.71de3a556c734p-19, 0x1.27e4fb7789f5cp-22, 0x1.ae64567f544e4p-26,
    0x1.1eed8eff8d898p-29, 0x1.6124613a86d09p-33};
__device__ static const double LOG_C[12] = {
    0x1.0000000000000p+1, 0x1.5555555555555p-1, 0x1.999999999999ap-2, 0x1.2492492492492p-2,
    0x1.c71c71c71c71cp-3, 0x1.745d1745d1746p-3, 0x1.3b13b13b13b14p-3, 0x1.1111111111111p-3,
    0x1.e1e1e1e1e1e1ep-4, 0x1.af286bca1af28p-4, 0x1.8618618618618p-4, 0x1.642c8590b2164p-4};
__device__ static const double COS_C[11] = {
    0x1.0000000000000p+0,  -0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10,
    0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37,
    0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62};
__device__ static const double SIN_C[11] = {
    0x1.0000000000000p+0,  -0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
    0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41,
    0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57, 0x1.71b8ef6dcf572p-66};
constexpr double LN2_HI = 0x1.62e42fee00000p-1;
constexpr double LN2_LO = 0x1.a39ef35793c76p-33;
constexpr double LN2 = 0x1.62e42fefa39efp-1;
constexpr double INV_LN2 = 0x1.71547652b82fep+0;
constexpr double TWO_PI = 0x1.921fb54442d18p+2;
constexpr double SQRT_HALF = 0x1.6a09e667f3bcdp-1;

__device__ __forceinline__ double horner(const double *c, int n, double x) {
#pragma clang fp contract(off)
  double p = c[n - 1];
  for (int k = n - 2; k >= 0; --k) {
    p = p * x;
    p = p + c[k];
  }
  return p;
}

__device__ inline double det_exp(double x) {
#pragma clang fp contract(off)
  if (x > 708.0) return __builtin_huge_val();
  if (x < -708.0) return 0.0;
  const double n = __builtin_rint(x * INV_LN2);
  double r = x - n * LN2_HI;
  r = r - n * LN2_LO;
  const double p = horner(EXP_C, 14, r);
  return __builtin_ldexp(p, (int)n);
}

__device__ inline double det_log(double u) {
#pragma clang fp contract(off)
  int e;
  double m = __builtin_frexp(u, &e);
  if (m < SQRT_HALF) {
    m = m * 2.0;
    e = e - 1;
  }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double s2 = s * s;
  const double lm = s * horner(LOG_C, 12, s2);
  return (double)e * LN2 + lm;
}

__device__ inline double det_cos2pi(double t) {
#pragma clang fp contract(off)
  if (t >= 0.5) t = 1.0 - t;
  const bool neg = t > 0.25;
  if (neg) t = 0.5 - t;
  const bool use_sin = t > 0.125;
  const double t2 = use_sin ? 0.25 - t : t;
  const double x = TWO_PI * t2;
  const double xx = x * x;
  const double r = use_sin ? x * horner(SIN_C, 11, xx) : horner(COS_C, 11, xx);
  return neg ? -r : r;
}

__device__ inline double det_normal(double u1, double u2) {
#pragma clang fp contract(off)
  return __builtin_sqrt(-2.0 * det_log(u1)) * det_cos2pi(u2);
}

__device__ inline float det_sigmoid32(float z) {
#pragma clang fp contract(off)
  const double e = det_exp(-(double)z);
  return (float)(1.0 / (1.0 + e));
}

}  // namespace detm
