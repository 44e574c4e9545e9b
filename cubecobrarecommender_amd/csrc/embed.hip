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
#include <algorithm>
#include <cstdlib>

#include "adam.hpp"
#include "common.hpp"
#include "xt.hpp"

// build knobs (A/B builds: CCREC_EXTRA_FLAGS=-D..., a tagged library; the library reads no
// environment): the gather / scatter variants below default to the measured-fastest ones
#ifndef CCREC_GATHER2
#define CCREC_GATHER2 48
#endif
#ifndef CCREC_GATHER_XCDW
#define CCREC_GATHER_XCDW 44
#endif
#ifndef CCREC_GATHER_XCD
#define CCREC_GATHER_XCD 44
#endif
#ifndef CCREC_GATHER_U
#define CCREC_GATHER_U 8
#endif
#ifndef CCREC_SCATTER_U
#define CCREC_SCATTER_U 8
#endif

// dev-only timing hook (tools/micro/eg_probe.hip defines it); compiled out of the library
#ifndef EG_PROBE
#define EG_PROBE(k)
#endif

namespace {

// EPL consecutive elements of one table row -> fp32, with the widest aligned vector loads.
template <typename T, int EPL>
__device__ __forceinline__ void load_row(const T *__restrict__ p, float (&v)[EPL]) {
  constexpr int BYTES = EPL * (int)sizeof(T);
  if constexpr (BYTES % 16 == 0) {
#pragma unroll
    for (int q = 0; q < BYTES / 16; ++q) {
      const uint4 u = reinterpret_cast<const uint4 *>(p)[q];
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (sizeof(T) == 2) {
          v[q * 8 + 2 * e] = __uint_as_float(w[e] << 16);
          v[q * 8 + 2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
        } else {
          v[q * 4 + e] = __uint_as_float(w[e]);
        }
      }
    }
  } else if constexpr (BYTES == 8) {
    const uint2 u = *reinterpret_cast<const uint2 *>(p);
    if constexpr (sizeof(T) == 2) {
      v[0] = __uint_as_float(u.x << 16);
      v[1] = __uint_as_float(u.x & 0xFFFF0000u);
      v[2] = __uint_as_float(u.y << 16);
      v[3] = __uint_as_float(u.y & 0xFFFF0000u);
    } else {
      v[0] = __uint_as_float(u.x);
      v[1] = __uint_as_float(u.y);
    }
  } else {
#pragma unroll
    for (int e = 0; e < EPL; ++e) v[e] = DT<T>::ld(p + e);
  }
}

// Forward: 4 waves per cube row, wave w sums the w-th quarter of the row's (sorted) card list
// with U row loads in flight per lane; the four partials are added in wave order (deterministic).
constexpr int GW = 4;
// E1 backward: waves per W1 row (measured: 2 -> 49 us, 4 -> 46, 8 -> 62, 16 -> 130 at cfg 2).
#ifndef CCREC_SCATTER_GW
#define CCREC_SCATTER_GW 4
#endif
constexpr int SGW = CCREC_SCATTER_GW;

// The row's index list is staged in LDS first (one coalesced read), so each batch of U row
// loads costs one dependent global round trip instead of two.
constexpr int GIDX = 2048;

template <typename T, int EPL, int U>
__global__ __launch_bounds__(256) void gather_kernel(const T *__restrict__ table,
                                                     const float *__restrict__ bias, int d, int R,
                                                     const int32_t *__restrict__ x_cnt,
                                                     const int32_t *__restrict__ x_idx, int x_cap,
                                                     T *__restrict__ out) {
  __shared__ float part[GW - 1][64 * EPL];
  __shared__ int32_t ls[GIDX];
  const int row = blockIdx.x;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = lane * EPL;
  float acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
  const int n = x_cnt[row];
  const int q = (n + GW - 1) / GW;
  const int i0 = min(n, w * q), i1 = min(n, i0 + q);
  const int32_t *__restrict__ glst = x_idx + (int64_t)row * x_cap;
  const bool staged = n <= GIDX;
  if (staged)
    for (int t = threadIdx.x; t < n; t += 256) ls[t] = glst[t];
  __syncthreads();
  const int32_t *lst = staged ? ls : glst;
  int i = i0;
  for (; i + U <= i1; i += U) {
    int j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = lst[i + u];
    float v[U][EPL];
#pragma unroll
    for (int u = 0; u < U; ++u) load_row<T, EPL>(table + (int64_t)j[u] * d + c0, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] += v[u][e];
  }
  for (; i < i1; ++i) {
    float v[EPL];
    load_row<T, EPL>(table + (int64_t)lst[i] * d + c0, v);
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[e] += v[e];
  }
  if (w > 0) {
#pragma unroll
    for (int e = 0; e < EPL; ++e) part[w - 1][c0 + e] = acc[e];
  }
  __syncthreads();
  if (w == 0) {
    T *o = out + (int64_t)row * d + c0;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      float v = acc[e];
#pragma unroll
      for (int p = 0; p < GW - 1; ++p) v += part[p][c0 + e];
      v += bias[c0 + e];
      DT<T>::st(o + e, v > 0.f ? v : 0.f);
    }
  }
}

__global__ __launch_bounds__(256) void xt_transpose_kernel(const uint32_t *__restrict__ xb, int V,
                                                           uint32_t *__restrict__ xt, int xt_rows) {
  xt_transpose_block(xb, V, xt, xt_rows, blockIdx.x);
}

// Forward, bf16 d = 256: each lane loads 16 B (8 columns) so one wave load instruction fetches TWO
// table rows (half-wave h takes list entries of parity h) — twice the bytes in flight per
// instruction; GWN waves per cube, U loads in flight per lane.  Partial sums: lane halves
// (shuffle), then waves in order through LDS — deterministic.
typedef __attribute__((ext_vector_type(4))) uint32_t g_u32x4;
template <int GWN, int U>
__global__ __launch_bounds__(64 * GWN) void gather2_kernel(const bf16_t *__restrict__ table,
                                                          const float *__restrict__ bias, int R,
                                                          const int32_t *__restrict__ x_cnt,
                                                          const int32_t *__restrict__ x_idx, int x_cap,
                                                          bf16_t *__restrict__ out, const void *warm,
                                                          int64_t warm_bytes, int64_t *state, int64_t bpe,
                                                          const uint32_t *__restrict__ xb, int V,
                                                          uint32_t *__restrict__ xt, int xt_rows) {
  const int nxt = xt ? (((V + 31) >> 5) + XT_TJ - 1) / XT_TJ : 0;
  if ((int)blockIdx.x < nxt) {  // blocks 0..nxt-1: the xt transpose (short; dispatched first, they
    xt_transpose_block(xb, V, xt, xt_rows, (int)blockIdx.x);  // run beside the latency-bound gather)
    return;
  }
  if (state && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the previous step's counters
    state[0] += 1;
    state[1] += 1;
    if (state[1] >= bpe) {
      state[1] = 0;
      state[2] += 1;
    }
  }
  constexpr int D = 256;
  __shared__ __attribute__((aligned(16))) float part[GWN][D];
  __shared__ int32_t ls[GIDX];
  const int row = (int)blockIdx.x - nxt;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int c0 = (lane & 31) * 8;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int n = x_cnt[row];
  const int q = ((n + GWN - 1) / GWN + 1) & ~1;  // even chunks: pairs never straddle waves
  const int i0 = min(n, w * q), i1 = min(n, i0 + q);
  const int32_t *__restrict__ glst = x_idx + (int64_t)row * x_cap;
  const bool staged = n <= GIDX;
  if (staged)
    for (int t = threadIdx.x; t < n; t += 64 * GWN) ls[t] = glst[t];
  __syncthreads();
  const int32_t *lst = staged ? ls : glst;
  int i = i0;
  for (; i + 2 * U <= i1; i += 2 * U) {
    int j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = lst[i + 2 * u + h];
    g_u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const g_u32x4 *>(table + (int64_t)j[u] * D + c0);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += __uint_as_float(v[u][e] << 16);
        acc[2 * e + 1] += __uint_as_float(v[u][e] & 0xFFFF0000u);
      }
  }
  for (; i + h < i1; i += 2) {
    const g_u32x4 v = *reinterpret_cast<const g_u32x4 *>(table + (int64_t)lst[i + h] * D + c0);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] += __uint_as_float(v[e] << 16);
      acc[2 * e + 1] += __uint_as_float(v[e] & 0xFFFF0000u);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], 32);
  if (h == 0) {
    *reinterpret_cast<float4 *>(&part[w][c0]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4 *>(&part[w][c0 + 4]) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
  __syncthreads();
  if (threadIdx.x < D / 8) {
    const int c = threadIdx.x * 8;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = part[0][c + e];
#pragma unroll
      for (int p = 1; p < GWN; ++p) v += part[p][c + e];
      v += bias[c + e];
      o[e] = v > 0.f ? v : 0.f;
    }
    g_u32x4 pk;
#pragma unroll
    for (int e = 0; e < 4; ++e) pk[e] = (uint32_t)f2bf(o[2 * e]) | ((uint32_t)f2bf(o[2 * e + 1]) << 16);
    *reinterpret_cast<g_u32x4 *>(out + (int64_t)row * D + c) = pk;
  }
  l2_warm(warm, warm_bytes, row, R);  // the tower forward's packed weights (gather blocks only)
}

// Forward, bf16 d = 256, column slices dealt to XCDs.  gather2 gives every block all 256 columns
// of its row, so each XCD's 4 MB L2 sees the whole 11 MB W1 table (48 MB fetched beyond L2 per
// step for an 11 MB table).  Here block b runs on XCD b % 8 (round-robin dispatch) and owns the
// 64-column slice (b % 8) & 3 of row 2 (b / 8) + (b % 8) / 4: an XCD only ever reads one 128-B
// line of each W1 row (2.8 MB of the table, L2-resident).  A wave load fetches the slice of 8
// cards (8 lanes x 16 B each); the 8 card groups are added lane-wise by xor shuffles, the waves
// in order through LDS (deterministic).
constexpr int GX_NS = 4, GX_COLS = 256 / GX_NS;  // slices per row, columns per slice
template <int GWN, int U>
__global__ __launch_bounds__(64 * GWN) void gather_xcd_kernel(const bf16_t *__restrict__ table,
                                                             const float *__restrict__ bias, int R,
                                                             const int32_t *__restrict__ x_cnt,
                                                             const int32_t *__restrict__ x_idx, int x_cap,
                                                             bf16_t *__restrict__ out, const void *warm,
                                                             int64_t warm_bytes, int64_t *state, int64_t bpe) {
  if (state && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the previous step's counters
    state[0] += 1;
    state[1] += 1;
    if (state[1] >= bpe) {
      state[1] = 0;
      state[2] += 1;
    }
  }
  constexpr int D = 256;
  __shared__ __attribute__((aligned(16))) float part[GWN][GX_COLS];
  __shared__ int32_t ls[GIDX];
  const int xcd = (int)blockIdx.x & 7;
  const int row = 2 * ((int)blockIdx.x >> 3) + (xcd >> 2);
  const int slice = xcd & (GX_NS - 1);
  if (row < R) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 3;
    const int c0 = slice * GX_COLS + (lane & 7) * 8;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const int n = x_cnt[row];
    const int q = ((n + GWN - 1) / GWN + 7) & ~7;  // chunks of whole 8-card groups
    const int i0 = min(n, w * q), i1 = min(n, i0 + q);
    const int32_t *__restrict__ glst = x_idx + (int64_t)row * x_cap;
    const bool staged = n <= GIDX;
    if (staged)
      for (int t = threadIdx.x; t < n; t += 64 * GWN) ls[t] = glst[t];
    __syncthreads();
    const int32_t *lst = staged ? ls : glst;
    int i = i0;
    for (; i + 8 * U <= i1; i += 8 * U) {
      int j[U];
#pragma unroll
      for (int u = 0; u < U; ++u) j[u] = lst[i + 8 * u + g];
      g_u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const g_u32x4 *>(table + (int64_t)j[u] * D + c0);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] += __uint_as_float(v[u][e] << 16);
          acc[2 * e + 1] += __uint_as_float(v[u][e] & 0xFFFF0000u);
        }
    }
    for (; i < i1; i += 8) {
      if (i + g < i1) {
        const g_u32x4 v = *reinterpret_cast<const g_u32x4 *>(table + (int64_t)lst[i + g] * D + c0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] += __uint_as_float(v[e] << 16);
          acc[2 * e + 1] += __uint_as_float(v[e] & 0xFFFF0000u);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc[e] += __shfl_xor(acc[e], 8);
      acc[e] += __shfl_xor(acc[e], 16);
      acc[e] += __shfl_xor(acc[e], 32);
    }
    if (g == 0) {
      const int c = (lane & 7) * 8;
      *reinterpret_cast<float4 *>(&part[w][c]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4 *>(&part[w][c + 4]) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
    __syncthreads();
    if (threadIdx.x < GX_COLS / 8) {
      const int c = threadIdx.x * 8;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = part[0][c + e];
#pragma unroll
        for (int p = 1; p < GWN; ++p) v += part[p][c + e];
        v += bias[slice * GX_COLS + c + e];
        o[e] = v > 0.f ? v : 0.f;
      }
      g_u32x4 pk;
#pragma unroll
      for (int e = 0; e < 4; ++e) pk[e] = (uint32_t)f2bf(o[2 * e]) | ((uint32_t)f2bf(o[2 * e + 1]) << 16);
      *reinterpret_cast<g_u32x4 *>(out + (int64_t)row * D + slice * GX_COLS + c) = pk;
    }
  }
  l2_warm(warm, warm_bytes, (int)blockIdx.x, (int)gridDim.x);  // the tower forward's packed weights
}

// Forward, bf16 d = 512 / 1024: the same XCD column slicing with all eight XCDs on one row.  Block
// nxt8 + b runs on XCD b % 8 and owns the (d / 8)-column slice b % 8 of row b / 8 (d = 1024: 256 B
// of each W1 row per XCD, 5.6 MB of the 45 MB table; gather_kernel gave every block whole rows, so
// every XCD's L2 streamed the whole table).  LPC = d / 64 lanes x 16 B cover one card's slice, a
// wave load fetches G = 64 / LPC cards; the card groups are added lane-wise by xor shuffles, the
// waves in order through LDS (deterministic).  The first nxt8 blocks (a multiple of 8, so the
// slice mapping is unchanged) bit-transpose F's x rows into the W1-gradient bitmask when xt is
// given, and the last block advances the step counters: no separate launches for either.
template <int D, int GWN, int U>
__global__ __launch_bounds__(64 * GWN) void gather_xcdw_kernel(const bf16_t *__restrict__ table,
                                                              const float *__restrict__ bias,
                                                              const int32_t *__restrict__ x_cnt,
                                                              const int32_t *__restrict__ x_idx, int x_cap,
                                                              bf16_t *__restrict__ out, int64_t *state, int64_t bpe,
                                                              const uint32_t *__restrict__ xb, int V,
                                                              uint32_t *__restrict__ xt, int xt_rows, int nxt8) {
  constexpr int SW = D / 8, LPC = SW / 8, G = 64 / LPC;
  if ((int)blockIdx.x < nxt8) {
    const int nxt = xt ? (((V + 31) >> 5) + XT_TJ - 1) / XT_TJ : 0;
    if ((int)blockIdx.x < nxt) xt_transpose_block(xb, V, xt, xt_rows, (int)blockIdx.x);
    return;
  }
  if (state && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the previous step's counters
    state[0] += 1;
    state[1] += 1;
    if (state[1] >= bpe) {
      state[1] = 0;
      state[2] += 1;
    }
  }
  __shared__ __attribute__((aligned(16))) float part[GWN][SW];
  __shared__ int32_t ls[GIDX];
  const int slice = (int)blockIdx.x & 7;
  const int row = ((int)blockIdx.x - nxt8) >> 3;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane / LPC;
  const int cl = (lane % LPC) * 8, c0 = slice * SW + cl;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int n = x_cnt[row];
  const int q = ((n + GWN - 1) / GWN + G - 1) / G * G;  // chunks of whole G-card groups
  const int i0 = min(n, w * q), i1 = min(n, i0 + q);
  const int32_t *__restrict__ glst = x_idx + (int64_t)row * x_cap;
  const bool staged = n <= GIDX;
  if (staged)
    for (int t = threadIdx.x; t < n; t += 64 * GWN) ls[t] = glst[t];
  __syncthreads();
  const int32_t *lst = staged ? ls : glst;
  int i = i0;
  for (; i + G * U <= i1; i += G * U) {
    int j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = lst[i + G * u + g];
    g_u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const g_u32x4 *>(table + (int64_t)j[u] * D + c0);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += __uint_as_float(v[u][e] << 16);
        acc[2 * e + 1] += __uint_as_float(v[u][e] & 0xFFFF0000u);
      }
  }
  for (; i < i1; i += G) {
    if (i + g < i1) {
      const g_u32x4 v = *reinterpret_cast<const g_u32x4 *>(table + (int64_t)lst[i + g] * D + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += __uint_as_float(v[e] << 16);
        acc[2 * e + 1] += __uint_as_float(v[e] & 0xFFFF0000u);
      }
    }
  }
#pragma unroll
  for (int o = LPC; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], o);
  if (g == 0) {
    *reinterpret_cast<float4 *>(&part[w][cl]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4 *>(&part[w][cl + 4]) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
  __syncthreads();
  if (threadIdx.x < LPC) {
    const int c = threadIdx.x * 8;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = part[0][c + e];
#pragma unroll
      for (int p = 1; p < GWN; ++p) v += part[p][c + e];
      v += bias[slice * SW + c + e];
      o[e] = v > 0.f ? v : 0.f;
    }
    g_u32x4 pk;
#pragma unroll
    for (int e = 0; e < 4; ++e) pk[e] = (uint32_t)f2bf(o[2 * e]) | ((uint32_t)f2bf(o[2 * e + 1]) << 16);
    *reinterpret_cast<g_u32x4 *>(out + (int64_t)row * D + slice * SW + c) = pk;
  }
}

// Backward: 4 waves per W1 row (row V = the bias when bias_grad is given); wave w walks the w-th
// quarter of the row's bit words, collecting up to U set bits before issuing their dPre loads
// together (heavy Zipf rows have a set bit for nearly every batch row).  Partials added in wave order.
template <int EPL, int U>
__global__ __launch_bounds__(64 * SGW) void scatter_bwd_kernel(const float *__restrict__ dpre, int V,
                                                          int d, int R,
                                                          const uint32_t *xt,
                                                          float *__restrict__ grad,
                                                          float *__restrict__ bias_grad) {
  
  __shared__ float part[SGW - 1][64 * EPL];
  const int row = blockIdx.x;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int XW = (R + 31) >> 5;
  const int c0 = lane * EPL;
  float acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
  const uint32_t *bits = xt + (int64_t)row * XW;
  const int q = (XW + SGW - 1) / SGW;
  const int w0 = min(XW, w * q), w1 = min(XW, w0 + q);
  int pend[U];
  int np = 0;
  for (int wd = w0; wd < w1; ++wd) {
    uint32_t m = row == V ? (wd == XW - 1 && (R & 31) ? (1u << (R & 31)) - 1u : 0xFFFFFFFFu) : bits[wd];
    while (m) {
      // static-indexed shift register (a runtime-indexed array would live in scratch)
#pragma unroll
      for (int u = U - 1; u > 0; --u) pend[u] = pend[u - 1];
      pend[0] = (wd << 5) + __ffs(m) - 1;
      m &= m - 1;
      if (++np == U) {
        float v[U][EPL];
#pragma unroll
        for (int u = 0; u < U; ++u) load_row<float, EPL>(dpre + (int64_t)pend[u] * d + c0, v[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int e = 0; e < EPL; ++e) acc[e] += v[u][e];
        np = 0;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (u < np) {
      float v[EPL];
      load_row<float, EPL>(dpre + (int64_t)pend[u] * d + c0, v);
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] += v[e];
    }
  }
  // consume the bitmask: this wave is the only reader of words [w0, w1) of the row, and every
  // one of its loads above has been used, so clearing leaves xt zeroed for the next step's F
  if (row < V)
    for (int wd = w0 + lane; wd < w1; wd += 64) const_cast<uint32_t *>(bits)[wd] = 0u;
  if (w > 0) {
#pragma unroll
    for (int e = 0; e < EPL; ++e) part[w - 1][c0 + e] = acc[e];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int e = 0; e < EPL; ++e)
#pragma unroll
      for (int p = 0; p < SGW - 1; ++p) acc[e] += part[p][c0 + e];
    float *g = row == V ? bias_grad + c0 : grad + (int64_t)row * d + c0;
    if constexpr (EPL % 4 == 0) {
#pragma unroll
      for (int qq = 0; qq < EPL / 4; ++qq)
        reinterpret_cast<float4 *>(g)[qq] =
            make_float4(acc[4 * qq], acc[4 * qq + 1], acc[4 * qq + 2], acc[4 * qq + 3]);
    } else {
#pragma unroll
      for (int e = 0; e < EPL; ++e) g[e] = acc[e];
    }
  }
}

// Backward on bf16 MFMA (cc_embed_grad_mfma): dW1 = X^T dPre1 as a dense [V, R] x [R, d] product
// whose A operand is the transposed x bitmask itself — each lane's 8-k A fragment is one byte of
// the row's bit words expanded to bf16 0/1 in registers (exact), B = dPre1^T bf16 [d][RP] (written
// by the tower backward chain).  Every row costs the same (no Zipf-heavy row latency chain, no
// per-row dispatch); row V (with bias_grad) is the all-ones row: db1 = colsum dPre1.  A block owns
// EG_ROWS rows of W1 and all d columns, so it also clears the bit words it consumed.
constexpr int EG_ROWS = 64, EG_BK = 64;
constexpr int EG_XWMAX = 64;  // R <= 2048 (bit words per row staged in LDS: template XWM <= EG_XWMAX)

typedef __attribute__((ext_vector_type(4))) uint32_t eg_u32x4;  // ext vectors stay in VGPRs
__device__ __forceinline__ bf16x8_t expand_bits8(uint32_t b) {
  eg_u32x4 w;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = (((b >> (2 * i)) & 1u) * 0x3F80u) | (((b >> (2 * i + 1)) & 1u) * 0x3F800000u);
  return __builtin_bit_cast(bf16x8_t, w);
}

template <int NC, int XWM>
__global__ __launch_bounds__(256, 2) void embed_grad_mfma_kernel(const bf16_t *__restrict__ gT, int V,
                                                                int d, int R, int RP, uint32_t *xt,
                                                                float *__restrict__ grad,
                                                                float *__restrict__ bias_grad) {
  constexpr int CH = EG_BK / 8;                 // 16-B chunks per B row per K-tile
  constexpr int NCH = NC * CH / 256;            // chunks staged per thread
  constexpr int NJ = NC / 64;                   // 32-col accumulators per wave (2 x 2 waves)
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][NC * EG_BK];
  __shared__ uint32_t As[EG_ROWS][XWM + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, half = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int v0 = blockIdx.x * EG_ROWS;
  // R rows enter the product; RP is the B image's row stride (>= ceil64(R): the full-mode
  // regulariser's identity rows sit past R in the same image and are added separately)
  const int RPE = (R + 63) & ~63;
  const int XW = (R + 31) >> 5, XWP = RPE >> 5;
  EG_PROBE(0);
  // the block's bit words: every load issued before any store (one HBM round trip, not one per
  // word — the zeroing stores would otherwise order each next load behind them)
  constexpr int AS_Q = EG_ROWS * XWM / 256;
  uint32_t mv[AS_Q];
#pragma unroll
  for (int q = 0; q < AS_Q; ++q) {
    const int i = tid + 256 * q, r = i / XWP, w = i % XWP, v = v0 + r;
    mv[q] = 0u;
    if (i < EG_ROWS * XWP && w < XW) {
      if (v < V)
        mv[q] = xt[(int64_t)v * XW + w];
      else if (v == V && bias_grad)
        mv[q] = (w == XW - 1 && (R & 31)) ? (1u << (R & 31)) - 1u : 0xFFFFFFFFu;
    }
  }
#pragma unroll
  for (int q = 0; q < AS_Q; ++q) {
    const int i = tid + 256 * q, r = i / XWP, w = i % XWP, v = v0 + r;
    if (i < EG_ROWS * XWP) {
      if (w < XW && v < V) xt[(int64_t)v * XW + w] = 0u;  // consumed: the next step's F finds xt zeroed
      As[r][w] = mv[q];
    }
  }
  const int nk = RPE / EG_BK;
  const int arow = wm * 32 + (lane & 31);
  for (int nc0 = 0; nc0 < d; nc0 += NC) {
    f32x16_t acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    eg_u32x4 st[NCH];
#define EG_LOAD(KT)                                                                                   \
  _Pragma("unroll") for (int q = 0; q < NCH; ++q) {                                                   \
    const int c = tid + 256 * q, n = c / CH, ch = c % CH;                                             \
    st[q] = *reinterpret_cast<const eg_u32x4 *>(gT + (int64_t)(nc0 + n) * RP + (KT) * EG_BK + ch * 8); \
  }
#define EG_STORE(BUF)                                                                          \
  _Pragma("unroll") for (int q = 0; q < NCH; ++q) {                                            \
    const int c = tid + 256 * q, n = c / CH, ch = c % CH;                                      \
    *reinterpret_cast<eg_u32x4 *>(&Bs[BUF][n * EG_BK + ((ch ^ (n & (CH - 1))) * 8)]) = st[q];     \
  }
    EG_LOAD(0)
    __syncthreads();  // As visible; previous chunk's readers of Bs are done
    EG_STORE(0)
    __syncthreads();
    EG_PROBE(1);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) { EG_LOAD(kt + 1) }
      const bf16_t *bs = Bs[kt & 1];
#pragma unroll
      for (int kk = 0; kk < EG_BK / 16; ++kk) {
        const int k = kt * EG_BK + kk * 16 + 8 * half;
        const bf16x8_t a = expand_bits8((As[arow][k >> 5] >> (k & 31)) & 0xFFu);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = wn * (NC / 2) + j * 32 + (lane & 31);
          const bf16x8_t b = *reinterpret_cast<const bf16x8_t *>(bs + n * EG_BK + (((2 * kk + half) ^ (n & (CH - 1))) * 8));
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
        }
      }
      if (kt + 1 < nk) { EG_STORE((kt + 1) & 1) }
      __syncthreads();
      EG_PROBE(2 + kt);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = nc0 + wn * (NC / 2) + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int v = v0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (v < V)
          grad[(int64_t)v * d + col] = acc[j][r];
        else if (v == V && bias_grad)
          bias_grad[col] = acc[j][r];
      }
    }
  }
  EG_PROBE(15);
#undef EG_LOAD
#undef EG_STORE
}

// cc_embed_grad_packed: the same product with B fragments streamed from the packed transposed
// dPre1 image.  Wave w owns columns [64w, 64w + 64) for all EG_ROWS rows (2 x 2 accumulator
// tiles), so each B fragment is loaded once per block; A = the row's bit bytes expanded in
// registers (LDS bit words, as above).  EG_PU fragment pairs in flight per lane.
constexpr int EG_PU = 8;
template <int XWM>
__global__ __launch_bounds__(256, 2) void embed_grad_pk_kernel(const bf16_t *__restrict__ gP, int V, int R,
                                                              int RP, uint32_t *xt, float *__restrict__ grad,
                                                              float *__restrict__ bias_grad) {
  constexpr int D = 256;
  __shared__ uint32_t As[EG_ROWS][XWM + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5;
  const int v0 = blockIdx.x * EG_ROWS;
  const int RPE = (R + 63) & ~63;  // rows in the product; RP: the packed image's reduction stride
  const int XW = (R + 31) >> 5, XWP = RPE >> 5;
  constexpr int AS_Q = EG_ROWS * XWM / 256;
  uint32_t mv[AS_Q];
#pragma unroll
  for (int q = 0; q < AS_Q; ++q) {
    const int i = tid + 256 * q, r = i / XWP, wd = i % XWP, v = v0 + r;
    mv[q] = 0u;
    if (i < EG_ROWS * XWP && wd < XW) {
      if (v < V)
        mv[q] = xt[(int64_t)v * XW + wd];
      else if (v == V && bias_grad)
        mv[q] = (wd == XW - 1 && (R & 31)) ? (1u << (R & 31)) - 1u : 0xFFFFFFFFu;
    }
  }
  // the first fragments fly while the bit words are staged
  const bf16_t *b0 = gP + ((int64_t)(2 * w) * (RP / 16) * 64 + lane) * 8;
  const bf16_t *b1 = gP + ((int64_t)(2 * w + 1) * (RP / 16) * 64 + lane) * 8;
  const int nk = RPE / 16;
  bf16x8_t f0[EG_PU], f1[EG_PU];
#pragma unroll
  for (int u = 0; u < EG_PU; ++u)
    if (u < nk) {
      f0[u] = *reinterpret_cast<const bf16x8_t *>(b0 + u * 512);
      f1[u] = *reinterpret_cast<const bf16x8_t *>(b1 + u * 512);
    }
#pragma unroll
  for (int q = 0; q < AS_Q; ++q) {
    const int i = tid + 256 * q, r = i / XWP, wd = i % XWP, v = v0 + r;
    if (i < EG_ROWS * XWP) {
      if (wd < XW && v < V) xt[(int64_t)v * XW + wd] = 0u;  // consumed: the next step's F finds xt zeroed
      As[r][wd] = mv[q];
    }
  }
  __syncthreads();
  f32x16_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int r0 = lane & 31, r1 = 32 + (lane & 31);
  for (int j0 = 0; j0 < nk; j0 += EG_PU) {
#pragma unroll
    for (int u = 0; u < EG_PU; ++u) {
      const int j = j0 + u;
      if (j >= nk) break;
      const int k = 16 * j + 8 * half;
      const bf16x8_t a0 = expand_bits8((As[r0][k >> 5] >> (k & 31)) & 0xFFu);
      const bf16x8_t a1 = expand_bits8((As[r1][k >> 5] >> (k & 31)) & 0xFFu);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, f0[u], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, f1[u], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, f0[u], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, f1[u], acc[1][1], 0, 0, 0);
      if (j + EG_PU < nk) {  // refill the slot just consumed
        f0[u] = *reinterpret_cast<const bf16x8_t *>(b0 + (j + EG_PU) * 512);
        f1[u] = *reinterpret_cast<const bf16x8_t *>(b1 + (j + EG_PU) * 512);
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int col = 64 * w + 32 * b + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int v = v0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (v < V)
          grad[(int64_t)v * D + col] = acc[a][b][r];
        else if (v == V && bias_grad)
          bias_grad[col] = acc[a][b][r];
      }
    }
}

// cc_embed_grad_cs: the same product by COLUMN SLICE.  The row-tile kernels above give every block
// all d columns, so every block re-reads the whole dPre1 image (256 KB at R = 512) from L2 —
// 88 MB for the step at ~70 GB/s per CU, and their 344 blocks leave the 2-block CUs on the
// critical path.  Here block (row chunk rc, slice cs) owns 32 columns: it stages its slice of
// dPre1 (nk = ceil64(R)/16 MFMA B fragments, 1 KB each) in LDS once, and each of its 8 waves
// takes 32-row tiles of the chunk: the tile's bit words go straight into registers (a lane holds
// its row's XWM words), A fragments come from a byte LUT in LDS (256 values x 16 lane copies,
// 16 B each: one conflict-free ds_read_b128) instead of ~20 VALU bit tricks per fragment.  Same MFMA k
// order per tile as the kernels above: the same fp32 results.  The chunk's xt words are cleared
// by the last of its slice blocks to finish (a ticket per chunk, reset by that block: no spin, no
// extra launch).
constexpr int CS_NT = 512;                     // 8 waves, ~one block per CU
// config 5's instance (XWM = 32, R = 1024, TF Adam in the epilogue): tiles per wave, the Adam-operand
// prefetch and the k-steps per fragment group trade registers (build-time A/B knobs)
#ifndef EG_TPW32
#define EG_TPW32 3
#endif
#ifndef EG_PF_XWM
#define EG_PF_XWM 16
#endif
#ifndef EG_CSG32
#define EG_CSG32 4
#endif
constexpr int cs_tpw(int xwm, bool adam = false) {  // tiles per wave (registers)
  return xwm <= 16 ? 3 : xwm <= 32 ? (adam ? EG_TPW32 : 3) : 1;
}
// byte -> 8 bf16 (16 B) LUT lane copies: fewer where the LDS is short (R > 512 with the Adam
// epilogue's re-layout tiles, R > 1024): 2-way bank conflicts at 8 copies
constexpr int cs_lut_copies(int xwm, bool adam) { return xwm <= 16 ? 16 : xwm <= 32 ? (adam ? 8 : 16) : 4; }
constexpr int cs_lut_bytes(int xwm, bool adam) { return 256 * 16 * cs_lut_copies(xwm, adam); }
__device__ __forceinline__ uint4 byte_bf16(uint32_t e) {  // 8 bits -> 8 bf16 of 1.0 / 0.0
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (((e >> (2 * i)) & 1u) ? 0x3F80u : 0u) | (((e >> (2 * i + 1)) & 1u) ? 0x3F800000u : 0u);
  return make_uint4(w[0], w[1], w[2], w[3]);
}
// the W1 Adam epilogue's p / m / v streams (read and written once per step): cache policy.
// Non-temporal measured slower (W1 kernel 32 -> 41 us in the BCE step, r03 A/B): default.
#ifndef EG_ADAM_NT
#define EG_ADAM_NT 0
#endif
__device__ __forceinline__ cc_adam::f32x4_t eg_ld(const cc_adam::f32x4_t *q) {
  if constexpr (EG_ADAM_NT) return __builtin_nontemporal_load(q);
  else return *q;
}
__device__ __forceinline__ void eg_st(cc_adam::f32x4_t *q, cc_adam::f32x4_t v) {
  if constexpr (EG_ADAM_NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}
// ADAM: TF Adam on W1 in the tile epilogue (one process: the gradient is final here) — p, m, v
// stream through once, the bf16 shadow is rewritten, the W1 gradient is never stored; the bias
// row's gradient still goes to bias_grad for the main Adam launch
#ifndef EG_PREFETCH
#define EG_PREFETCH 1
#endif
struct CsAdam {
  float *p, *m, *v;      // W1 rows of the flat fp32 buffers ([V][d])
  bf16_t *shadow;        // W1 rows of the bf16 shadow
  const int64_t *state;  // device step counters: t = state[0] + 1 (cc_adam_dense's t)
  float lr, b1, b2, eps;
};
// REG: the sampled regulariser's identity rows by index instead of by bit.  Row B + i of the batch
// (i < nreg) is the one-card row {rid[i]} (generator.py:47-61: x_reg = identity rows of the reg
// draws), so in the bit matrix a W1 row holds at most a handful of the nreg reg bits and most of
// the product's reg k-steps multiply an all-zero A fragment.  With REG the bit matrix covers the B
// cube rows only (the product's K = B: the XWM = 16 instance at B = 512 instead of XWM = 32), and each
// tile adds the reg k-steps whose A fragment is not all zero for its 32 rows — found from rid (in
// LDS), A fragments built from rid compares, B fragments loaded from the same dPre1 image (k-step
// k0 + ks) — in ascending order after the cube k-steps: the MFMA sequence of the full-K product
// minus its all-zero k-steps, i.e. the same fp32 results.  The bias row (all rows) takes every
// reg k-step.
struct CsReg {
  const int32_t *rid;  // [nreg] cards of the reg rows (absolute card ids; -1: a padding row)
  int nreg;            // <= CS_REG_MAX (512)
  int k0;              // the first reg k-step in the dPre1 image (= B / 16)
  int card0;           // card of this launch's W1 row 0 (a row chunk's first row)
};
constexpr int CS_REG_MAX = 512;   // (one 32-bit mask of reg k-steps per tile)
// (Measured and dropped, round 6, tools/micro/eg_reg_probe.hip: per wave, a tile of popular cards
// or the bias tile takes many reg k-steps and ends its wave ~10 us after the rest.  Neither the
// chunks interleaved over the blocks (+14 us on the + KL step: the bias tile then shares a wave
// with two full tiles; BCE +1, config 5 +20-35 us, profiles/r06y_w1_tstride_ab.txt) nor the reg
// k-steps' B fragments staged in LDS (with half the LUT copies to make room: + KL +3 us,
// profiles/r06z_w1_reg_lds_ab.txt) nor each batch's rid reads / A bytes / LUT reads / MFMAs issued
// phase by phase (neutral, profiles/r06g_w1_reg_pipe_ab.txt) beat the code below.)

template <bool PK, int XWM, bool VEC, bool ADAM, bool REG = false>
__global__ __launch_bounds__(CS_NT, 1) void embed_grad_cs_kernel(const bf16_t *__restrict__ gsrc, int V, int d, int R,
                                                            int RP, int tpc, uint32_t *xt,
                                                            float *__restrict__ grad,
                                                            float *__restrict__ bias_grad, uint32_t *tickets,
                                                            CsAdam ad, CsReg rg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5;
  const int nsl = d >> 5, cs = blockIdx.x % nsl, rc = blockIdx.x / nsl;
  const int RPE = (R + 63) & ~63, nk = RPE >> 4;
  const int XW = (R + 31) >> 5;  // words per xt row; the product runs over XWM words (zeros past XW)
  const int rows_total = V + (bias_grad ? 1 : 0);
  const int NTL = (rows_total + 31) >> 5;
  const int t0 = rc * tpc, nt = min(NTL, t0 + tpc) - t0;
  const int v0 = 32 * t0;
  EG_PROBE(0);
  constexpr int LC = cs_lut_copies(XWM, ADAM);
  bf16_t *Bs = reinterpret_cast<bf16_t *>(smem);                  // fragment j at (j * 64 + lane) * 8
  unsigned char *lut = smem + (size_t)2 * XWM * 1024;             // [256 values][16 copies] x 16 B
  float *tx = reinterpret_cast<float *>(lut + cs_lut_bytes(XWM, ADAM));  // ADAM: per-wave 32 x 36 tiles
  // REG: the reg rows' cards, padded with -1 to a multiple of 512 entries
  int32_t *rl = reinterpret_cast<int32_t *>(reinterpret_cast<unsigned char *>(tx) + (ADAM ? (CS_NT / 64) * 32 * 36 * 4 : 0));
  // ---- every global read first: the bit words of all the wave's tiles (wave w takes tiles w,
  // w + 8, ... of the chunk; a lane holds its row's XWM words per tile), then the B slice and LUT
  // (every global load below is unconditional — clamped address, then a select — so the
  // compiler's vmcnt waits stay counted: a load behind a branch made it drain to zero, which
  // serialised the staging loads and the next tile's bit prefetch)
  auto load_bits = [&](int t, uint32_t (&wd)[XWM]) {
    const int v = v0 + 32 * t + (lane & 31);  // this lane's A row
    const bool real = t < nt && v < V;
    const uint32_t *src = xt + (int64_t)(real ? v : 0) * XW;
    if constexpr (VEC) {  // XW % 4 == 0: 16-B loads
#pragma unroll
      for (int q = 0; q < XWM / 4; ++q) {
        const uint4 x4 = *reinterpret_cast<const uint4 *>(src + 4 * min(q, XW / 4 - 1));
        wd[4 * q] = x4.x;
        wd[4 * q + 1] = x4.y;
        wd[4 * q + 2] = x4.z;
        wd[4 * q + 3] = x4.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < XWM; ++q) wd[q] = src[min(q, XW - 1)];
    }
    const bool brow = t < nt && v == V && bias_grad;  // the bias row: every batch row
#pragma unroll
    for (int q = 0; q < XWM; ++q) {
      const uint32_t bm = (q == XW - 1 && (R & 31)) ? (1u << (R & 31)) - 1u : 0xFFFFFFFFu;
      wd[q] = q >= XW ? 0u : real ? wd[q] : brow ? bm : 0u;
    }
  };
  constexpr int NW = CS_NT / 64;
  constexpr int TPW = cs_tpw(XWM, ADAM);  // tiles per wave (the host sizes tpc <= NW * TPW)
  uint32_t wds[TPW][XWM];
#pragma unroll
  for (int i = 0; i < TPW; ++i) load_bits(w + NW * i, wds[i]);
  // the B slice: 2 XWM fragments (those past nk are zero), a compile-time count per thread
  constexpr int NBT = 2 * XWM * 64 / CS_NT;
  {
    uint4 v[NBT];
    const uint4 *bsrc = reinterpret_cast<const uint4 *>(gsrc + (int64_t)cs * (RP / 16) * 512);
#pragma unroll
    for (int u = 0; u < NBT; ++u) {
      const int f = u * CS_NT + tid, fc = min(f, nk * 64 - 1);
      if constexpr (PK) {  // packed transposed dPre1: the slice's fragments are one contiguous run
        v[u] = bsrc[fc];
      } else {  // dPre1^T [d][RP]: fragment (j, lane) = 8 consecutive rows of column 32 cs + (lane & 31)
        const int j = fc >> 6, ln = fc & 63;
        v[u] = *reinterpret_cast<const uint4 *>(gsrc + (int64_t)(32 * cs + (ln & 31)) * RP + 16 * j + 8 * (ln >> 5));
      }
    }
#pragma unroll
    for (int u = 0; u < NBT; ++u) {
      const int f = u * CS_NT + tid;
      reinterpret_cast<uint4 *>(Bs)[f] = (f >> 6) < nk ? v[u] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  for (int e = tid; e < 256 * LC; e += CS_NT) reinterpret_cast<uint4 *>(lut)[e] = byte_bf16((uint32_t)(e / LC));
  if constexpr (REG) {   // (unconditional loads, clamped index: counted waits stay exact)
    constexpr int RQ = CS_REG_MAX / CS_NT;
    const int nr512 = (rg.nreg + 511) & ~511;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int i = tid + CS_NT * q;
      const int32_t c = rg.rid[min(i, rg.nreg - 1)];
      if (i < nr512) rl[i] = i < rg.nreg ? c : -1;
    }
  }
  EG_PROBE(1);
  __syncthreads();  // (its release fence: every load of the block, bit words included, has returned)
  EG_PROBE(2);
  // the chunk's ticket now, before any store of this block: the last of the chunk's nsl slice
  // blocks to get here clears the chunk's xt words at its end; the atomic's return is read there
  // (it was issued before the stores, so that wait does not drain them)
  uint32_t tk = 0u;
  if (tid == 0 && tickets) tk = __hip_atomic_fetch_add(&tickets[rc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // ---- tiles
  // the A fragment of a byte: one ds_read_b128 from this lane's copy (lane & 15: the 16 lanes a
  // b128 read serves per cycle hit 16 distinct bank quads, whatever their bytes) — full rate even
  // at one or two waves per SIMD, where 8-B LDS reads run at a fifth of it
  const unsigned char *lutl = lut + (lane % LC) * 16;
  const uint32_t sh = 8u * (uint32_t)half;
  // XWM = 16 (R <= 512, the headline shape): the wave keeps the whole B slice in 128 VGPRs, read
  // from LDS once — the tile loop then reads only its A fragments from LDS (at two 1-KB LDS reads
  // per MFMA the LDS array, not the MFMA, set the pace)
  constexpr bool BREG = XWM == 16 && !ADAM;  // (the Adam epilogue needs those registers)
  bf16x8_t breg[BREG ? 2 * XWM : 1];
  if constexpr (BREG) {
#pragma unroll
    for (int k = 0; k < 2 * XWM; ++k) breg[k] = *reinterpret_cast<const bf16x8_t *>(Bs + (k * 64 + lane) * 8);
  }
  float alpha = 0.f, omb1 = 0.f, omb2 = 0.f;
  if constexpr (ADAM) {  // cc_adam::range's constants, same expressions
    const float tt = (float)(ad.state[0] + 1);
    const float b1p = powf(ad.b1, tt), b2p = powf(ad.b2, tt);
    alpha = ad.lr * sqrtf(1.f - b2p) / (1.f - b1p);
    omb1 = 1.f - ad.b1;
    omb2 = 1.f - ad.b2;
  }
  // Adam operands of a tile's 16 elements per lane (unconditional: a clamped row, stored only for
  // real rows), double-buffered: tile i + 1's are issued before tile i's epilogue, so its load
  // latency runs under that epilogue and tile i + 1's MFMAs (EG_PREFETCH, R <= 512: the taller
  // instances have no registers left for the second buffer; else before the MFMAs)
  // (the Adam epilogue works on the tile re-laid through LDS: instruction g covers tile rows
  // 8 g .. 8 g + 7, lane l row 8 g + (l >> 3), columns 4 (l & 7) .. +3 — eight whole 128-B lines
  // per wave instruction instead of 32 partial ones)
  constexpr bool PF = ADAM && EG_PREFETCH && XWM <= EG_PF_XWM;
  constexpr int NBUF = PF ? 2 : 1;
  cc_adam::f32x4_t AP[NBUF][ADAM ? 4 : 1], AM[NBUF][ADAM ? 4 : 1], AV[NBUF][ADAM ? 4 : 1];
  auto issue_adam = [&](int t, int b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int vg = v0 + 32 * t + 8 * g + (lane >> 3);
      const int64_t rb = (int64_t)(vg < V ? vg : V - 1) * d + 32 * cs + 4 * (lane & 7);
      AP[b][g] = eg_ld(reinterpret_cast<const cc_adam::f32x4_t *>(ad.p + rb));
      AM[b][g] = eg_ld(reinterpret_cast<const cc_adam::f32x4_t *>(ad.m + rb));
      AV[b][g] = eg_ld(reinterpret_cast<const cc_adam::f32x4_t *>(ad.v + rb));
    }
  };
  if constexpr (PF) {
    if (w < nt) issue_adam(w, 0);
  }
  // REG: dPre1 fragment of reg k-step ks (clamped: an unconditional load)
  auto reg_bfrag = [&](int ks) -> bf16x8_t {
    const int k = rg.k0 + max(ks, 0);
    if constexpr (PK)
      return *reinterpret_cast<const bf16x8_t *>(gsrc + ((int64_t)cs * (RP / 16) * 64 + (int64_t)k * 64 + lane) * 8);
    else
      return *reinterpret_cast<const bf16x8_t *>(gsrc + (int64_t)(32 * cs + (lane & 31)) * RP + 16 * k + 8 * half);
  };
  auto tile = [&](int t, const uint32_t (&wd)[XWM], int b, int tn) {
    const int vr = v0 + 32 * t + (lane & 31);
    // REG: the reg k-steps with an entry in this tile (km: bit ks), the first RPF of them prefetched
    // under the cube k-steps (the bias tile takes all of them)
    constexpr int RPF = 2, NKW = REG ? CS_REG_MAX / 512 : 1;
    uint32_t km[NKW];
    bf16x8_t rb[REG ? RPF : 1];
    int rks[REG ? RPF : 1];
    const int tcard = rg.card0 + v0 + 32 * t;                  // the tile's first card
    const bool btile = bias_grad && v0 + 32 * t <= V && V < v0 + 32 * t + 32;   // (wave-uniform)
    auto next_k = [&]() -> int {   // pop the lowest relevant k-step (-1: none left); wave-uniform
#pragma unroll
      for (int q = 0; q < NKW; ++q)
        if (km[q]) {
          const int k = 32 * q + __builtin_ctz(km[q]);
          km[q] &= km[q] - 1u;
          return k;
        }
      return -1;
    };
    if constexpr (REG) {
#pragma unroll
      for (int q = 0; q < NKW; ++q) {
        km[q] = 0u;
        if (512 * q < rg.nreg) {
          const int i0 = 512 * q + 8 * lane;   // lane l: entries i0 .. i0 + 7 = half of k-step i0 / 16
          const int4 e0 = *reinterpret_cast<const int4 *>(rl + i0), e1 = *reinterpret_cast<const int4 *>(rl + i0 + 4);
          const uint32_t u = (uint32_t)tcard;
          const bool hit = btile ? i0 < rg.nreg
                                 : ((uint32_t)e0.x - u < 32u) | ((uint32_t)e0.y - u < 32u) | ((uint32_t)e0.z - u < 32u) |
                                       ((uint32_t)e0.w - u < 32u) | ((uint32_t)e1.x - u < 32u) | ((uint32_t)e1.y - u < 32u) |
                                       ((uint32_t)e1.z - u < 32u) | ((uint32_t)e1.w - u < 32u);
          uint64_t x = __ballot(hit);
          x = (x | (x >> 1)) & 0x5555555555555555ull;   // lanes 2k, 2k + 1 -> bit 2k
          x = (x | (x >> 1)) & 0x3333333333333333ull;   // ... then gather the even bits
          x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
          x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
          x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
          x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
          km[q] = __builtin_amdgcn_readfirstlane((uint32_t)x);
        }
      }
#pragma unroll
      for (int u = 0; u < RPF; ++u) {
        rks[u] = next_k();
        rb[u] = reg_bfrag(rks[u]);
      }
    }
    if constexpr (ADAM && !PF) issue_adam(t, 0);
    cc_adam::f32x4_t(&ap)[ADAM ? 4 : 1] = AP[NBUF == 2 ? b : 0];
    cc_adam::f32x4_t(&am)[ADAM ? 4 : 1] = AM[NBUF == 2 ? b : 0];
    cc_adam::f32x4_t(&av)[ADAM ? 4 : 1] = AV[NBUF == 2 ? b : 0];
    f32x16_t acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // A fragment of k-step k (word k/2, half-word k%2, this lane's byte): one LUT read; B: one
    // ds_read_b128 of the staged slice.  Groups of CS_G k-steps: the next group's 2 CS_G reads are
    // issued (sched_barrier) before this group's MFMAs, so the LDS latency runs under them.  The
    // B address is made opaque per tile so the compiler does not hoist the whole slice into VGPRs.
    constexpr int CS_G = (XWM == 32 && ADAM) ? EG_CSG32 : 4, NG = 2 * XWM / CS_G;
    uint32_t boff = (uint32_t)lane * 16u;  // byte offset of this lane's fragment slot in Bs
    asm volatile("" : "+v"(boff));
    auto fetch = [&](int g, bf16x8_t (&da)[CS_G], bf16x8_t (&db)[CS_G]) {
#pragma unroll
      for (int u = 0; u < CS_G; ++u) {
        const int k = CS_G * g + u;
        const uint32_t s = 16u * (uint32_t)(k & 1) + sh;
        da[u] = *reinterpret_cast<const bf16x8_t *>(lutl + __builtin_amdgcn_ubfe(wd[k >> 1], s, 8) * (16 * LC));
        if constexpr (BREG)
          db[u] = breg[k];
        else
          db[u] = *reinterpret_cast<const bf16x8_t *>(reinterpret_cast<const unsigned char *>(Bs) + boff + k * 1024);
      }
    };
    bf16x8_t af[2][CS_G], bf[2][CS_G];
    fetch(0, af[0], bf[0]);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) fetch(g + 1, af[(g + 1) & 1], bf[(g + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < CS_G; ++u)  // operands swapped: acc = (dW1 tile)^T, see below
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[g & 1][u], af[g & 1][u], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (REG) {   // the tile's reg k-steps, ascending: the prefetched RPF, then batches of RB
      const int card = tcard + (lane & 31);
      const bool brl = bias_grad && vr == V;   // this lane's row is the bias row
      auto reg_mfma = [&](int ks, const bf16x8_t &bfr) {
        const int i0 = 16 * ks + 8 * half;
        const int4 e0 = *reinterpret_cast<const int4 *>(rl + i0), e1 = *reinterpret_cast<const int4 *>(rl + i0 + 4);
        const int ev[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
        uint32_t byte = 0u;
#pragma unroll
        for (int e = 0; e < 8; ++e) byte |= (brl ? i0 + e < rg.nreg : ev[e] == card) ? 1u << e : 0u;
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t *>(lutl + byte * (16 * LC));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr, a, acc, 0, 0, 0);
      };
#pragma unroll
      for (int u = 0; u < RPF; ++u)
        if (rks[u] >= 0) reg_mfma(rks[u], rb[u]);
      // the rest (the bias tile: every reg k-step; tiles of popular cards) RB loads in flight at a
      // time — the k-loop's fragment registers are free here
      constexpr int RB = 8;
      int k = next_k();
      while (k >= 0) {   // (wave-uniform)
        bf16x8_t bq[RB];
        int kq[RB];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
          kq[u] = k;
          bq[u] = reg_bfrag(k);   // (clamped: an unconditional load)
          k = next_k();
        }
#pragma unroll
        for (int u = 0; u < RB; ++u)
          if (kq[u] >= 0) reg_mfma(kq[u], bq[u]);
      }
    }
    // With the dPre1 fragments as the MFMA's A operand and the bit fragments as its B operand (the
    // same registers), lane l holds W1 row v0 + 32 t + (l & 31) and the slice's columns
    // 8 g + 4 (l >> 5) .. +3, g = 0..3: four 16-B stores per lane instead of sixteen 4-B ones.
    if constexpr (PF) {
      if (tn < nt) issue_adam(tn, b ^ 1);  // the next tile's operands fly during this epilogue
    }
    if constexpr (ADAM) {
      float *T = tx + w * (32 * 36);  // this wave's 32 x 32 tile, row pitch 36 floats
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4 *>(T + (lane & 31) * 36 + 8 * g + 4 * half) =
            make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int rr = 8 * g + (lane >> 3), c0 = 32 * cs + 4 * (lane & 7);
        const int vg = v0 + 32 * t + rr;
        const float4 q = *reinterpret_cast<const float4 *>(T + rr * 36 + 4 * (lane & 7));
        if (vg < V) {
          float pe[4] = {ap[g][0], ap[g][1], ap[g][2], ap[g][3]}, me[4] = {am[g][0], am[g][1], am[g][2], am[g][3]};
          float ve[4] = {av[g][0], av[g][1], av[g][2], av[g][3]};
          const float ge[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) cc_adam::elem(pe[e], me[e], ve[e], ge[e], alpha, omb1, omb2, ad.eps);
          const int64_t o = (int64_t)vg * d + c0;
          eg_st(reinterpret_cast<cc_adam::f32x4_t *>(ad.p + o), cc_adam::f32x4_t{pe[0], pe[1], pe[2], pe[3]});
          eg_st(reinterpret_cast<cc_adam::f32x4_t *>(ad.m + o), cc_adam::f32x4_t{me[0], me[1], me[2], me[3]});
          eg_st(reinterpret_cast<cc_adam::f32x4_t *>(ad.v + o), cc_adam::f32x4_t{ve[0], ve[1], ve[2], ve[3]});
          ushort4 sh;
          sh.x = f2bf(pe[0]);
          sh.y = f2bf(pe[1]);
          sh.z = f2bf(pe[2]);
          sh.w = f2bf(pe[3]);
          *reinterpret_cast<ushort4 *>(ad.shadow + o) = sh;
        } else if (vg == V && bias_grad) {
          *reinterpret_cast<float4 *>(bias_grad + c0) = q;
        }
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = 32 * cs + 8 * g + 4 * half;
        const float4 q = make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
        if (vr < V)
          *reinterpret_cast<float4 *>(grad + (int64_t)vr * d + c0) = q;
        else if (vr == V && bias_grad)
          *reinterpret_cast<float4 *>(bias_grad + c0) = q;
      }
    }
  };
#pragma unroll
  for (int i = 0; i < TPW; ++i)
    if (w + NW * i < nt) tile(w + NW * i, wds[i], i & 1, w + NW * (i + 1));
  EG_PROBE(3);
  if (tickets) {  // (no tickets: the caller rewrites every xt word before the next use)
    if (tid == 0) last = tk == (uint32_t)(nsl - 1);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // LDS only: no store drain
    if (last) {
      const int vend = min(V, v0 + 32 * nt);
      for (int64_t i = (int64_t)v0 * XW + tid; i < (int64_t)vend * XW; i += CS_NT) xt[i] = 0u;
      if (tid == 0) __hip_atomic_store(&tickets[rc], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  EG_PROBE(15);
}

// launch geometry of cc_embed_grad_cs: 32-row tiles per chunk and the LDS size
void cs_plan(int V, int d, int R, bool bias, int &tpc, int &nrc, size_t &lds, bool adam = false) {
  const int RPE = (R + 63) & ~63;
  const int NTL = (V + (bias ? 1 : 0) + 31) / 32;
  const int xwm = RPE / 32 <= 16 ? 16 : RPE / 32 <= 32 ? 32 : 64;  // the kernel's XWM
  const int nsl = d / 32;
  // ~one block per CU (the slice is staged once per block), at most cs_tpw tiles per wave
  nrc = std::max(std::max(1, std::min(NTL, 256 / nsl)), (int)cdiv(NTL, (CS_NT / 64) * cs_tpw(xwm, adam)));
  // more blocks than CUs (d = 1024: 29 chunks x 32 slices = 928): whole rounds of 256 blocks, so
  // the last round is not a fraction of the chip holding the whole launch (1024 blocks of 22 tiles
  // instead of 928 of 24)
  if (nrc * nsl > 256 && 256 % nsl == 0) nrc = (int)cdiv(nrc, 256 / nsl) * (256 / nsl);
  tpc = (int)cdiv(NTL, nrc);
  nrc = (int)cdiv(NTL, tpc);
  lds = (size_t)2 * xwm * 1024 + cs_lut_bytes(xwm, adam) + (adam ? (size_t)(CS_NT / 64) * 32 * 36 * 4 : 0);
}

}  // namespace

extern "C" int32_t cc_embed_grad_cs_tickets(int32_t V, int32_t d, int32_t R) {
  if (V <= 0 || d < 32 || R <= 0) return 0;
  int tpc, nrc, nrc_adam;
  size_t lds;
  cs_plan(V, d, R, true, tpc, nrc, lds);
  cs_plan(V, d, R, true, tpc, nrc_adam, lds, true);  // (the Adam instance may chunk finer)
  return std::max(nrc, nrc_adam);
}

static int embed_grad_cs_launch(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                                uint32_t *xt_bits, float *grad, float *bias_grad, uint32_t *tickets,
                                const CsAdam *ad, void *stream, const CsReg *rg = nullptr) {
  int tpc, nrc;
  size_t lds;
  cs_plan(V, d, R, bias_grad != nullptr, tpc, nrc, lds, ad != nullptr);
  if (rg) lds += (size_t)((rg->nreg + 511) & ~511) * 4;
  CC_REQUIRE(lds <= 160 * 1024 - 64, "cc_embed_grad_cs: R too large for the LDS stage");
  const dim3 grid((unsigned)(nrc * (d / 32)));
  const int xw = ((R + 63) & ~63) / 32;  // bit words per row in the product
  const bool vec = ((R + 31) / 32) % 4 == 0;  // xt rows 16-B aligned
  const CsAdam a = ad ? *ad : CsAdam{};
  const CsReg r = rg ? *rg : CsReg{};
  hipStream_t s = as_stream(stream);
#define CS_LAUNCH(PKV, XWMV, VECV, ADV)                                                                          \
  do {                                                                                                           \
    if (rg)                                                                                                      \
      hipLaunchKernelGGL((embed_grad_cs_kernel<PKV, XWMV, VECV, ADV, true>), grid, dim3(CS_NT), lds, s,          \
                         (const bf16_t *)dpre, V, d, R, ld_t, tpc, xt_bits, grad, bias_grad, tickets, a, r);     \
    else                                                                                                         \
      hipLaunchKernelGGL((embed_grad_cs_kernel<PKV, XWMV, VECV, ADV>), grid, dim3(CS_NT), lds, s,                \
                         (const bf16_t *)dpre, V, d, R, ld_t, tpc, xt_bits, grad, bias_grad, tickets, a, r);     \
  } while (0)
#define CS_LAUNCH2(XWMV, ADV)                                                                 \
  if (packed) {                                                                               \
    if (vec) CS_LAUNCH(true, XWMV, true, ADV); else CS_LAUNCH(true, XWMV, false, ADV);        \
  } else {                                                                                    \
    if (vec) CS_LAUNCH(false, XWMV, true, ADV); else CS_LAUNCH(false, XWMV, false, ADV);      \
  }
  if (ad) {
    if (xw <= 16) { CS_LAUNCH2(16, true) } else if (xw <= 32) { CS_LAUNCH2(32, true) } else { CS_LAUNCH2(64, true) }
  } else {
    if (xw <= 16) { CS_LAUNCH2(16, false) } else if (xw <= 32) { CS_LAUNCH2(32, false) } else { CS_LAUNCH2(64, false) }
  }
#undef CS_LAUNCH2
#undef CS_LAUNCH
  CC_LAUNCH_CHECK("embed_grad_cs_kernel");
  return CC_OK;
}

extern "C" int cc_embed_grad_cs(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                                uint32_t *xt_bits, float *grad, float *bias_grad, uint32_t *tickets, void *stream) {
  CC_REQUIRE(dpre && xt_bits && grad, "cc_embed_grad_cs: null pointer");
  CC_REQUIRE((((uintptr_t)grad | (uintptr_t)bias_grad) & 15) == 0, "cc_embed_grad_cs: grad / bias_grad 16-B aligned");
  CC_REQUIRE(d % 32 == 0 && d >= 32 && d <= 4096, "cc_embed_grad_cs: d must be a multiple of 32");
  CC_REQUIRE(V > 0 && R > 0 && R <= 2048, "cc_embed_grad_cs: V > 0, R in 1..2048");
  CC_REQUIRE(ld_t % 64 == 0 && ld_t >= R && ((uintptr_t)dpre % 16) == 0,
             "cc_embed_grad_cs: ld_t must be a multiple of 64 covering R, dPre1 image 16-B aligned");
  return embed_grad_cs_launch(dpre, packed, V, d, R, ld_t, xt_bits, grad, bias_grad, tickets, nullptr, stream);
}

extern "C" int cc_embed_grad_cs_adam(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R,
                                     int32_t ld_t, uint32_t *xt_bits, float *bias_grad, uint32_t *tickets, float *p,
                                     float *m, float *v, uint16_t *shadow, const int64_t *state, float lr,
                                     float beta1, float beta2, float eps, void *stream) {
  CC_REQUIRE(dpre && xt_bits && p && m && v && shadow && state, "cc_embed_grad_cs_adam: null pointer");
  CC_REQUIRE((((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)bias_grad) & 15) == 0 &&
                 ((uintptr_t)shadow & 7) == 0,
             "cc_embed_grad_cs_adam: p, m, v, bias_grad 16-B aligned, shadow 8-B aligned");
  CC_REQUIRE(d % 32 == 0 && d >= 32 && d <= 4096, "cc_embed_grad_cs_adam: d must be a multiple of 32");
  CC_REQUIRE(V > 0 && R > 0 && R <= 2048, "cc_embed_grad_cs_adam: V > 0, R in 1..2048");
  CC_REQUIRE(ld_t % 64 == 0 && ld_t >= R && ((uintptr_t)dpre % 16) == 0,
             "cc_embed_grad_cs_adam: ld_t must be a multiple of 64 covering R, dPre1 image 16-B aligned");
  const CsAdam ad{p, m, v, (bf16_t *)shadow, state, lr, beta1, beta2, eps};
  return embed_grad_cs_launch(dpre, packed, V, d, R, ld_t, xt_bits, nullptr, bias_grad, tickets, &ad, stream);
}

static const char *cs_reg_check(const int32_t *reg_idx, int32_t nreg, int32_t reg_k0, int32_t R, int32_t ld_t) {
  if (!reg_idx || nreg < 1 || nreg > CS_REG_MAX) return "reg_idx non-null, nreg in 1..512";
  if (reg_k0 < 0 || 16 * reg_k0 < R || 16 * (reg_k0 + (nreg + 15) / 16) > ld_t)
    return "reg rows past the product's rows and inside the dPre1 image (16 reg_k0 >= R, 16 (reg_k0 + ceil(nreg / 16)) <= ld_t)";
  return nullptr;
}

extern "C" int cc_embed_grad_cs_reg(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                                    uint32_t *xt_bits, float *grad, float *bias_grad, uint32_t *tickets,
                                    const int32_t *reg_idx, int32_t nreg, int32_t reg_k0, int32_t card0, void *stream) {
  CC_REQUIRE(dpre && xt_bits && grad, "cc_embed_grad_cs_reg: null pointer");
  CC_REQUIRE((((uintptr_t)grad | (uintptr_t)bias_grad) & 15) == 0, "cc_embed_grad_cs_reg: grad / bias_grad 16-B aligned");
  CC_REQUIRE(d % 32 == 0 && d >= 32 && d <= 4096, "cc_embed_grad_cs_reg: d must be a multiple of 32");
  CC_REQUIRE(V > 0 && R > 0 && R <= 2048 && card0 >= 0, "cc_embed_grad_cs_reg: V > 0, R in 1..2048, card0 >= 0");
  CC_REQUIRE(ld_t % 64 == 0 && ld_t >= R && ((uintptr_t)dpre % 16) == 0,
             "cc_embed_grad_cs_reg: ld_t must be a multiple of 64 covering R, dPre1 image 16-B aligned");
  const char *e = cs_reg_check(reg_idx, nreg, reg_k0, R, ld_t);
  CC_REQUIRE(!e, e);
  const CsReg rg{reg_idx, nreg, reg_k0, card0};
  return embed_grad_cs_launch(dpre, packed, V, d, R, ld_t, xt_bits, grad, bias_grad, tickets, nullptr, stream, &rg);
}

extern "C" int cc_embed_grad_cs_adam_reg(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R,
                                         int32_t ld_t, uint32_t *xt_bits, float *bias_grad, uint32_t *tickets, float *p,
                                         float *m, float *v, uint16_t *shadow, const int64_t *state, float lr,
                                         float beta1, float beta2, float eps, const int32_t *reg_idx, int32_t nreg,
                                         int32_t reg_k0, void *stream) {
  CC_REQUIRE(dpre && xt_bits && p && m && v && shadow && state, "cc_embed_grad_cs_adam_reg: null pointer");
  CC_REQUIRE((((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)bias_grad) & 15) == 0 &&
                 ((uintptr_t)shadow & 7) == 0,
             "cc_embed_grad_cs_adam_reg: p, m, v, bias_grad 16-B aligned, shadow 8-B aligned");
  CC_REQUIRE(d % 32 == 0 && d >= 32 && d <= 4096, "cc_embed_grad_cs_adam_reg: d must be a multiple of 32");
  CC_REQUIRE(V > 0 && R > 0 && R <= 2048, "cc_embed_grad_cs_adam_reg: V > 0, R in 1..2048");
  CC_REQUIRE(ld_t % 64 == 0 && ld_t >= R && ((uintptr_t)dpre % 16) == 0,
             "cc_embed_grad_cs_adam_reg: ld_t must be a multiple of 64 covering R, dPre1 image 16-B aligned");
  const char *e = cs_reg_check(reg_idx, nreg, reg_k0, R, ld_t);
  CC_REQUIRE(!e, e);
  const CsAdam ad{p, m, v, (bf16_t *)shadow, state, lr, beta1, beta2, eps};
  const CsReg rg{reg_idx, nreg, reg_k0, 0};
  return embed_grad_cs_launch(dpre, packed, V, d, R, ld_t, xt_bits, nullptr, bias_grad, tickets, &ad, stream, &rg);
}

extern "C" int cc_embed_gather_fwd_warm(int32_t dtype, const void *table, const float *bias, int32_t V,
                                        int32_t d, int32_t R, const int32_t *x_cnt,
                                        const int32_t *x_idx, int32_t x_cap, void *out,
                                        const void *warm, int64_t warm_bytes, int64_t *state,
                                        int64_t bpe, void *stream);

extern "C" int cc_embed_grad_packed(const void *dpre_p, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                                    uint32_t *xt_bits, float *grad, float *bias_grad, void *stream) {
  CC_REQUIRE(dpre_p && xt_bits && grad, "cc_embed_grad_packed: null pointer");
  CC_REQUIRE(d == 256, "cc_embed_grad_packed: d must be 256");
  CC_REQUIRE(R > 0 && R <= 32 * EG_XWMAX, "cc_embed_grad_packed: R must be 1..2048");
  CC_REQUIRE(ld_t % 64 == 0 && ld_t >= R && ((uintptr_t)dpre_p % 16) == 0,
             "cc_embed_grad_packed: ld_t must be a multiple of 64 covering R, image 16-B aligned");
  const int rows = bias_grad ? V + 1 : V;
  const dim3 grid((unsigned)cdiv(rows, EG_ROWS));
  if (R <= 1024)
    hipLaunchKernelGGL((embed_grad_pk_kernel<32>), grid, dim3(256), 0, as_stream(stream),
                       (const bf16_t *)dpre_p, V, R, ld_t, xt_bits, grad, bias_grad);
  else
    hipLaunchKernelGGL((embed_grad_pk_kernel<64>), grid, dim3(256), 0, as_stream(stream),
                       (const bf16_t *)dpre_p, V, R, ld_t, xt_bits, grad, bias_grad);
  CC_LAUNCH_CHECK("embed_grad_pk_kernel");
  return CC_OK;
}

namespace {
// Full-mode regulariser rows are one-hot identity rows: their W1 gradient is dPre1 itself, row by
// row (rows of W1 touched once each: plain read-modify-write, no atomics).  Block b handles rows
// [64b, 64b+64) for all d columns and writes its column sums to partial[b][d]; the bias gradient
// adds them in block order (deterministic).
constexpr int ID_ROWS = 64;
// 256 threads: d/4 threads per row (float4 columns), 1024/d rows per pass; every load of the
// block's rows is issued before the read-modify-writes (the per-row chain was latency-bound)
__global__ __launch_bounds__(256) void embed_identity_add_kernel(const float *__restrict__ dpre, int n, int d,
                                                                 int lo, int round_bf16,
                                                                 float *__restrict__ grad,
                                                                 float *__restrict__ partial) {
  __shared__ float4 red[256];
  const int tpr = d >> 2, rpp = 256 / tpr;
  const int q = threadIdx.x % tpr, rr = threadIdx.x / tpr;
  const int r0 = blockIdx.x * ID_ROWS, r1 = min(n, r0 + ID_ROWS);
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int rb = r0 + rr; rb < r1; rb += 4 * rpp) {
    float4 v[4], g[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = rb + u * rpp;
      if (r < r1) {
        v[u] = reinterpret_cast<const float4 *>(dpre + (int64_t)r * d)[q];
        g[u] = reinterpret_cast<const float4 *>(grad + (int64_t)(lo + r) * d)[q];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = rb + u * rpp;
      if (r < r1) {
        float4 x = v[u];
        if (round_bf16) x = make_float4(bf2f(f2bf(x.x)), bf2f(f2bf(x.y)), bf2f(f2bf(x.z)), bf2f(f2bf(x.w)));
        reinterpret_cast<float4 *>(grad + (int64_t)(lo + r) * d)[q] =
            make_float4(g[u].x + x.x, g[u].y + x.y, g[u].z + x.z, g[u].w + x.w);
        cs = make_float4(cs.x + x.x, cs.y + x.y, cs.z + x.z, cs.w + x.w);
      }
    }
  }
  red[threadIdx.x] = cs;
  __syncthreads();
  if (rr == 0) {  // column sums over the row groups in a fixed order
    float4 t = red[q];
    for (int k = 1; k < rpp; ++k) {
      const float4 o = red[k * tpr + q];
      t = make_float4(t.x + o.x, t.y + o.y, t.z + o.z, t.w + o.w);
    }
    reinterpret_cast<float4 *>(partial + (int64_t)blockIdx.x * d)[q] = t;
  }
}

// bias_grad[c] += sum_b partial[b][c]: 4 waves per 64 columns, wave w sums a contiguous quarter of
// the partials (8 loads in flight), then the quarters are added in wave order
__global__ __launch_bounds__(256) void embed_identity_bias_kernel(const float *__restrict__ partial, int nb,
                                                                  int d, float *__restrict__ bias_grad) {
  __shared__ float red[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + lane;
  const int per = (nb + 3) / 4, b0 = min(nb, w * per), b1 = min(nb, b0 + per);
  float s = 0.f;
  if (c < d) {
    int b = b0;
    for (; b + 8 <= b1; b += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = partial[(int64_t)(b + u) * d + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += partial[(int64_t)b * d + c];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < d) bias_grad[c] += ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}
}  // namespace

extern "C" size_t cc_embed_identity_ws(int32_t n, int32_t d) {
  return (size_t)cdiv(n, ID_ROWS) * (size_t)d * sizeof(float);
}

extern "C" int cc_embed_identity_add(int32_t dtype, const float *dpre, int32_t n, int32_t d, int32_t lo,
                                     float *grad, float *bias_grad, float *partial, void *stream) {
  CC_REQUIRE(dpre && grad && partial, "cc_embed_identity_add: null pointer");
  CC_REQUIRE(n >= 0 && d >= 64 && d <= 1024 && (d & (d - 1)) == 0 && lo >= 0, "cc_embed_identity_add: bad n/d/lo");
  if (n == 0) return CC_OK;
  const int nb = (int)cdiv(n, ID_ROWS);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(embed_identity_add_kernel, dim3(nb), dim3(256), 0, s, dpre, n, d, lo,
                     dtype == CC_BF16 ? 1 : 0, grad, partial);
  CC_LAUNCH_CHECK("embed_identity_add_kernel");
  if (bias_grad) {
    hipLaunchKernelGGL(embed_identity_bias_kernel, dim3((unsigned)cdiv(d, 64)), dim3(256), 0, s, partial, nb, d,
                       bias_grad);
    CC_LAUNCH_CHECK("embed_identity_bias_kernel");
  }
  return CC_OK;
}

extern "C" int cc_embed_gather_fwd(int32_t dtype, const void *table, const float *bias, int32_t V,
                                   int32_t d, int32_t R, const int32_t *x_cnt,
                                   const int32_t *x_idx, int32_t x_cap, void *out, void *stream) {
  return cc_embed_gather_fwd_warm(dtype, table, bias, V, d, R, x_cnt, x_idx, x_cap, out, nullptr, 0, nullptr, 1,
                                  stream);
}

extern "C" int cc_embed_gather_fwd_warm(int32_t dtype, const void *table, const float *bias, int32_t V,
                                        int32_t d, int32_t R, const int32_t *x_cnt,
                                        const int32_t *x_idx, int32_t x_cap, void *out,
                                        const void *warm, int64_t warm_bytes, int64_t *state,
                                        int64_t bpe, void *stream) {
  return cc_embed_gather_fwd_xt(dtype, table, bias, V, d, R, x_cnt, x_idx, x_cap, out, warm, warm_bytes, state,
                                bpe, nullptr, nullptr, 0, stream);
}

extern "C" int cc_embed_gather_fwd_xt(int32_t dtype, const void *table, const float *bias, int32_t V,
                                      int32_t d, int32_t R, const int32_t *x_cnt,
                                      const int32_t *x_idx, int32_t x_cap, void *out,
                                      const void *warm, int64_t warm_bytes, int64_t *state,
                                      int64_t bpe, const uint32_t *x_bits, uint32_t *xt_bits, int32_t xt_rows,
                                      void *stream) {
  CC_REQUIRE(!state || bpe >= 1, "cc_embed_gather_fwd_warm: batches_per_epoch");
  CC_REQUIRE(!xt_bits || (x_bits && xt_rows >= 1 && xt_rows <= R),
             "cc_embed_gather_fwd_xt: xt_bits needs x_bits and 1 <= xt_rows <= R");
  constexpr int g2 = CCREC_GATHER2;    // build knob: 16-B lanes, two rows per load; waves x loads
  constexpr int gw = CCREC_GATHER_XCDW;  // build knob: XCD column-sliced gather at d = 512 / 1024 (0 = gather_kernel)
  const bool xcdw = dtype == CC_BF16 && (d == 512 || d == 1024) && gw > 0 && R > 0 && R <= 4096;
  if (state && !(dtype == CC_BF16 && d == 256 && g2 > 0) && !xcdw) {  // other kernels: a separate launch
    if (int rc = cc_state_advance(state, bpe, stream)) return rc;
    state = nullptr;
  }
  CC_REQUIRE(table && bias && x_cnt && x_idx && out, "cc_embed_gather_fwd: null pointer");
  CC_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "cc_embed_gather_fwd: d must be 64..1024, %64");
  CC_REQUIRE(V > 0 && R >= 0 && x_cap > 0, "cc_embed_gather_fwd: bad sizes");
  if (R == 0) return CC_OK;
  const dim3 grid((unsigned)R), block(256);
  const int nxt = xt_bits ? (int)cdiv((V + 31) / 32, XT_TJ) : 0;  // xt transpose blocks
  const int epl = d / 64;
  hipStream_t s = as_stream(stream);
  constexpr int gx = CCREC_GATHER_XCD;  // build knob: XCD column-sliced gather (0 = gather2); waves x loads
  // (tall R — the full-mode regulariser's |V| one-card identity rows — stays on gather2: a block
  // per 64-column slice of a one-card row is mostly overhead; measured 48 -> 121 us at R = 22,528)
  if (dtype == CC_BF16 && d == 256 && g2 > 0 && gx > 0 && !xt_bits && R <= 4096) {
    const dim3 gxg((unsigned)(cdiv(R, 2) * 8));
#define GX(GWN, U) \
  if (gx == GWN * 10 + U) hipLaunchKernelGGL((gather_xcd_kernel<GWN, U>), gxg, dim3(64 * GWN), 0, s, \
                                             (const bf16_t *)table, bias, R, x_cnt, x_idx, x_cap, (bf16_t *)out, \
                                             warm, warm_bytes, state, bpe); else
    GX(4, 4) GX(4, 8) GX(2, 4) GX(2, 8) GX(8, 4) GX(8, 2)
      return cc::fail(CC_ERR_UNSUPPORTED, "CCREC_GATHER_XCD: unknown variant (build knob)");
#undef GX
    CC_LAUNCH_CHECK("gather_xcd_kernel");
    return CC_OK;
  }
  if (xcdw) {
    const int nxt8 = (int)cdiv(nxt, 8) * 8;
    const dim3 gwg((unsigned)(nxt8 + 8 * R));
#define GW(D, GWN, U)                                                                                           \
  if (d == D && gw == GWN * 10 + U)                                                                             \
    hipLaunchKernelGGL((gather_xcdw_kernel<D, GWN, U>), gwg, dim3(64 * GWN), 0, s, (const bf16_t *)table, bias, \
                       x_cnt, x_idx, x_cap, (bf16_t *)out, state, bpe, x_bits, V, xt_bits, xt_rows, nxt8);        \
  else
    GW(512, 4, 4) GW(512, 2, 8) GW(512, 4, 8) GW(1024, 4, 4) GW(1024, 2, 8) GW(1024, 4, 8)
      return cc::fail(CC_ERR_UNSUPPORTED, "CCREC_GATHER_XCDW: unknown variant");
#undef GW
    CC_LAUNCH_CHECK("gather_xcdw_kernel");
    return CC_OK;
  }
  if (dtype == CC_BF16 && d == 256 && g2 > 0) {
#define G2(GWN, U) \
  if (g2 == GWN * 10 + U) hipLaunchKernelGGL((gather2_kernel<GWN, U>), dim3((unsigned)(R + nxt)), dim3(64 * GWN), 0, s, \
                                             (const bf16_t *)table, bias, R, x_cnt, x_idx, x_cap, (bf16_t *)out, \
                                             warm, warm_bytes, state, bpe, x_bits, V, xt_bits, xt_rows);
    G2(4, 4) G2(4, 8) G2(8, 4) G2(8, 8) G2(4, 6) G2(8, 6)
#undef G2
    CC_LAUNCH_CHECK("gather2_kernel");
    return CC_OK;
  }
  if (xt_bits) {
    hipLaunchKernelGGL(xt_transpose_kernel, dim3((unsigned)nxt), dim3(256), 0, s, x_bits, V, xt_bits, xt_rows);
    CC_LAUNCH_CHECK("xt_transpose_kernel");
  }
  constexpr int gu = CCREC_GATHER_U;  // build knob: row loads in flight per lane (bf16, d = 256);
  //                                     measured at cfg 2: 8 -> 328.5 us/step, 16 -> 337, 32 -> 341
  if (dtype == CC_BF16 && epl == 4 && (gu == 16 || gu == 32)) {
    if (gu == 16)
      hipLaunchKernelGGL((gather_kernel<bf16_t, 4, 16>), grid, block, 0, s, (const bf16_t *)table,
                         bias, d, R, x_cnt, x_idx, x_cap, (bf16_t *)out);
    else
      hipLaunchKernelGGL((gather_kernel<bf16_t, 4, 32>), grid, block, 0, s, (const bf16_t *)table,
                         bias, d, R, x_cnt, x_idx, x_cap, (bf16_t *)out);
    CC_LAUNCH_CHECK("gather_kernel");
    return CC_OK;
  }
#define GATHER_CASE(E)                                                                              \
  case E:                                                                                           \
    if (dtype == CC_BF16)                                                                           \
      hipLaunchKernelGGL((gather_kernel<bf16_t, E, 8>), grid, block, 0, s, (const bf16_t *)table, \
                         bias, d, R, x_cnt, x_idx, x_cap, (bf16_t *)out);                          \
    else                                                                                            \
      hipLaunchKernelGGL((gather_kernel<float, E, 8>), grid, block, 0, s, (const float *)table,   \
                         bias, d, R, x_cnt, x_idx, x_cap, (float *)out);                           \
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
                                    const uint32_t *xt_bits, float *grad, float *bias_grad,
                                    void *stream) {
  CC_REQUIRE(dpre && xt_bits && grad, "cc_embed_scatter_bwd: null pointer");
  CC_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "cc_embed_scatter_bwd: d must be 64..1024, %64");
  const dim3 grid((unsigned)(bias_grad ? V + 1 : V)), block(64 * SGW);
  hipStream_t s = as_stream(stream);
  constexpr int su = CCREC_SCATTER_U;  // build knob: dPre row loads in flight per lane (d = 256);
  //                                      measured at cfg 2: 8 -> 45.5 us, 16 -> 54.8
  if (d == 256 && su == 16) {
    hipLaunchKernelGGL((scatter_bwd_kernel<4, 16>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad, bias_grad);
    CC_LAUNCH_CHECK("scatter_bwd_kernel");
    return CC_OK;
  }
  switch (d / 64) {
    case 1: hipLaunchKernelGGL((scatter_bwd_kernel<1, 8>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad, bias_grad); break;
    case 2: hipLaunchKernelGGL((scatter_bwd_kernel<2, 8>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad, bias_grad); break;
    case 4: hipLaunchKernelGGL((scatter_bwd_kernel<4, 8>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad, bias_grad); break;
    case 8: hipLaunchKernelGGL((scatter_bwd_kernel<8, 8>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad, bias_grad); break;
    case 16: hipLaunchKernelGGL((scatter_bwd_kernel<16, 8>), grid, block, 0, s, dpre, V, d, R, xt_bits, grad, bias_grad); break;
    default: return cc::fail(CC_ERR_UNSUPPORTED, "cc_embed_scatter_bwd: d/64 must be a power of two");
  }
  CC_LAUNCH_CHECK("scatter_bwd_kernel");
  return CC_OK;
}

extern "C" int cc_embed_grad_mfma(const void *dpre_t, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                                  uint32_t *xt_bits, float *grad, float *bias_grad, void *stream) {
  CC_REQUIRE(dpre_t && xt_bits && grad, "cc_embed_grad_mfma: null pointer");
  CC_REQUIRE(d % 128 == 0 && d >= 128 && d <= 1024, "cc_embed_grad_mfma: d must be 128..1024, %128");
  CC_REQUIRE(R > 0 && R <= 32 * EG_XWMAX, "cc_embed_grad_mfma: R must be 1..2048");
  CC_REQUIRE(ld_t % EG_BK == 0 && ld_t >= R && ((uintptr_t)dpre_t % 16) == 0,
             "cc_embed_grad_mfma: ld_t must be a multiple of 64 covering R (zero padded), 16-B aligned");
  const int rows = bias_grad ? V + 1 : V;
  const dim3 grid((unsigned)cdiv(rows, EG_ROWS)), block(256);
  hipStream_t s = as_stream(stream);
#define EGM(NCC, XWMM)                                                                                 \
  hipLaunchKernelGGL((embed_grad_mfma_kernel<NCC, XWMM>), grid, block, 0, s, (const bf16_t *)dpre_t, V, d, R, \
                     ld_t, xt_bits, grad, bias_grad)
  if (d % 256 == 0) {
    if (R <= 1024) EGM(256, 32); else EGM(256, 64);
  } else {
    if (R <= 1024) EGM(128, 32); else EGM(128, 64);
  }
#undef EGM
  CC_LAUNCH_CHECK("embed_grad_mfma_kernel");
  return CC_OK;
}
