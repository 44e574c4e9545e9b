// Fused E/D towers on 32-row blocks (model.py:29-33 encoder Dense 256/128/64, :58-62 decoder Dense
// 128/256/d, both decoders) — forward and backward chains in ONE launch each instead of ~20 small
// GEMM launches.  Rows are independent through the towers, so a block owns RB = 32 rows of the
// batch and carries them through every layer with the activations in LDS; the weights (0.4 MB)
// stream from L2.  MFMA: v_mfma_f32_32x32x16_bf16 (bf16) / v_mfma_f32_32x32x2_f32 (fp32 parity).
//
// Forward layer  : out[32][N] = relu(X[32][K] W[K][N] + b);  A = X (LDS, row-major),
//                  B fragments from W^T [N][K] (global, k-contiguous) — cc_tower_transpose.
// Backward layer : dW_partial[K][N] = H^T G over the block's 32 rows (A = H^T, B = G from the
//                  transposed LDS images), db_partial = colsum G  -> slab[blk] (no atomics);
//                  dH[32][K] = G W^T (B fragments straight from W [K][N]) masked by H > 0.
// cc_tower_reduce sums the slabs in block order: deterministic dW/db for all 9 layers.
#include <algorithm>

#include "adam.hpp"
#include "common.hpp"
#include "mx8.hpp"
#include "noise_dev.hpp"
#include "xt.hpp"

// dev-only timing hook (tools/micro/tower_probe.hip defines it); compiled out of the library
#ifndef TOWER_PROBE
#define TOWER_PROBE(k)
#endif

namespace {

constexpr int RB = 32;   // rows per block
constexpr int NT = 256;  // 4 waves

struct TowerP {
  int d, B, R, maxw;
  const void *w[9];
  void *wt[9];
  const float *b[9];
  void *act[7];
  void *act6t;
  const void *gD3;
  void *gact[5];
  float *gpre1;
  void *gpre1t;  // optional bf16 dPre1^T [d][ceil64(R)]
  float *slab;
  int64_t slab_elems;
  float *gw[9];
  float *gb[9];
  const bf16_t *wpf[9];  // fragment-packed forward / backward weight images (cc_tower_args)
  const bf16_t *wpb[9];
  bf16_t *act6p, *act6tp;  // packed D3 operand images for cc_dec_bce_dw (fast forward only)
  bf16_t *hpt[6], *gpt[6];  // packed transposed H_i / G_i images for the dW kernel (or null)
  bf16_t *gpre1p;           // packed transposed dPre1 for cc_embed_grad_packed (or null)
  const uint32_t *xb;       // x row bitmasks -> xt (fast forward's extra blocks; or null)
  uint32_t *xt;
  int xt_V, xt_rows;
  uint8_t *d3q, *d3qs, *d3tq, *d3tqs;  // D3's MX-FP8 operand images (config 5; wide forward only, or null)
  const uint32_t *yb;       // y row bitmasks [B][y_VW] -> yimg (fast forward's extra blocks; or null)
  uint32_t *yimg;
  int y_VW;
  bool packed, dwpacked;
};

__host__ __device__ inline void chain_dims(int d, int i, int &K, int &N) {
  // K: d, 256, 128, 64, 128, 256;  N: 256, 128, 64, 128, 256, d  (no arrays: no scratch)
  K = i == 0 ? d : i == 1 ? 256 : i == 2 ? 128 : i == 3 ? 64 : i == 4 ? 128 : 256;
  N = i == 0 ? 256 : i == 1 ? 128 : i == 2 ? 64 : i == 3 ? 128 : i == 4 ? 256 : d;
}
__host__ __device__ inline int64_t slab_off(int d, int i) {  // chain layer i (0..5): kernel, bias
  int64_t o = 0;
  for (int j = 0; j < i; ++j) {
    int K, N;
    chain_dims(d, j, K, N);
    o += (int64_t)K * N + N;
  }
  return o;
}

template <typename T> struct TMma;
template <> struct TMma<bf16_t> {
  static constexpr int KM = 16;
  using frag = bf16x8_t;
  static __device__ __forceinline__ frag ld(const bf16_t *p, int kk, int half) {
    return *reinterpret_cast<const bf16x8_t *>(p + kk + 8 * half);
  }
  static __device__ __forceinline__ void mma(const frag &a, const frag &b, f32x16_t &c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct TMma<float> {
  static constexpr int KM = 2;
  using frag = float;
  static __device__ __forceinline__ frag ld(const float *p, int kk, int half) { return p[kk + half]; }
  static __device__ __forceinline__ void mma(const frag &a, const frag &b, f32x16_t &c) {
    c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// dPre1^T [d][ceil64(R)] (bf16): accumulator registers 4g..4g+3 hold 4 consecutive rows of column
// col, stored as one 8-byte word per g
__device__ __forceinline__ void gpre1t_store(const TowerP &p, int col, int r0, int lane, const bf16_t (&tt)[16]) {
  bf16_t *dt = reinterpret_cast<bf16_t *>(p.gpre1t) + (int64_t)col * ((p.R + 63) & ~63) + r0 + 4 * (lane >> 5);
#pragma unroll
  for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2 *>(dt + 8 * g) = *reinterpret_cast<const uint2 *>(&tt[4 * g]);
}

// C tile (32 rows x 32 cols starting at column n0) = A[32][K] (LDS row-major, lda) . Bt[n][K]
// (global, row n0+(lane&31) of a [N][K] k-contiguous matrix).  Loads for UB k-steps are issued
// before their MFMAs.
template <typename T>
__device__ __forceinline__ void tile_mm(const T *A, int lda, const T *__restrict__ Bt, int K, int n0,
                                        f32x16_t &acc) {
  using M = TMma<T>;
  constexpr int UB = 8;
  const int lane = threadIdx.x & 63, half = lane >> 5;
  const T *arow = A + (lane & 31) * lda;
  const T *brow = Bt + (int64_t)(n0 + (lane & 31)) * K;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  int kk = 0;
  for (; kk + UB * M::KM <= K; kk += UB * M::KM) {
    typename M::frag b[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) b[u] = M::ld(brow, kk + u * M::KM, half);
#pragma unroll
    for (int u = 0; u < UB; ++u) M::mma(M::ld(arow, kk + u * M::KM, half), b[u], acc);
  }
  for (; kk < K; kk += M::KM) M::mma(M::ld(arow, kk, half), M::ld(brow, kk, half), acc);
}

template <typename T>
__device__ __forceinline__ void lds_store_rows(T *Xr, int ldx, T *Xt, int ldt, int row, int col, float v) {
  T tv;
  DT<T>::st(&tv, v);
  Xr[row * ldx + col] = tv;
  if (Xt) Xt[col * ldt + row] = tv;
}

// copy a [32][W] block of a global [R][W] activation into LDS row-major (+ transposed) images
template <typename T>
__device__ void load_block(const T *__restrict__ g, int W, int r0, T *Xr, int ldx, T *Xt, int ldt) {
  constexpr int VW = 16 / sizeof(T);
  if (!Xt && W % VW == 0 && ldx % VW == 0) {
    // 16-B vectors: the block's rows are contiguous in global memory ([R][W] row-major)
    const int per = W / VW, nv = RB * per;
    const uint4 *src = reinterpret_cast<const uint4 *>(g + (int64_t)r0 * W);
    for (int i0 = 0; i0 < nv; i0 += 4 * NT) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + u * NT + (int)threadIdx.x < nv) v[u] = src[i0 + u * NT + threadIdx.x];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * NT + threadIdx.x;
        if (i < nv) *reinterpret_cast<uint4 *>(Xr + (i / per) * ldx + (i % per) * VW) = v[u];
      }
    }
    return;
  }
  for (int i = threadIdx.x; i < RB * W; i += NT) {
    const int row = i / W, col = i % W;
    const T v = g[(int64_t)(r0 + row) * W + col];
    Xr[row * ldx + col] = v;
    if (Xt) Xt[col * ldt + row] = v;
  }
}

// row-major block copy with a given block size (16-B vectors; W % 8 == 0, ldx % 8 == 0)
template <typename T, int THREADS>
__device__ void load_block_n(const T *__restrict__ g, int W, int r0, T *Xr, int ldx) {
  constexpr int VW = 16 / sizeof(T);
  const int per = W / VW, nv = RB * per;
  const uint4 *src = reinterpret_cast<const uint4 *>(g + (int64_t)r0 * W);
  for (int i = threadIdx.x; i < nv; i += THREADS)
    *reinterpret_cast<uint4 *>(Xr + (i / per) * ldx + (i % per) * VW) = src[i];
}

// transposed copy: Xt[col][row] = g[r0 + row][col] for the block's RB rows (16-B global loads)
template <typename T>
__device__ void load_block_t(const T *__restrict__ g, int W, int r0, T *Xt, int ldt) {
  constexpr int VW = 16 / sizeof(T);
  if (W % VW == 0) {
    const int per = W / VW, nv = RB * per;
    const uint4 *src = reinterpret_cast<const uint4 *>(g + (int64_t)r0 * W);
    for (int i0 = 0; i0 < nv; i0 += 4 * NT) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + u * NT + (int)threadIdx.x < nv) v[u] = src[i0 + u * NT + threadIdx.x];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * NT + threadIdx.x;
        if (i >= nv) continue;
        const int row = i / per, c0 = (i % per) * VW;
        const T *e = reinterpret_cast<const T *>(&v[u]);
#pragma unroll
        for (int q = 0; q < VW; ++q) Xt[(c0 + q) * ldt + row] = e[q];
      }
    }
    return;
  }
  for (int e = threadIdx.x; e < RB * W; e += NT) Xt[(e % W) * ldt + e / W] = g[(int64_t)(r0 + e / W) * W + e % W];
}

template <typename T>
__global__ __launch_bounds__(NT) void tower_fwd_kernel(TowerP p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ldx = p.maxw + 16 / (int)sizeof(T);
  T *X0 = reinterpret_cast<T *>(smem);
  T *X1 = X0 + RB * ldx;
  const int blk = blockIdx.x, r0 = blk * RB;
  const bool reg = r0 >= p.B;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  load_block<T>(reinterpret_cast<const T *>(p.act[0]), p.d, r0, X0, ldx, (T *)nullptr, 0);
  __syncthreads();
  T *xin = X0, *xout = X1;
  for (int i = 0; i < 6; ++i) {
    const int l = i < 3 ? i : i + (reg ? 3 : 0);  // layer index 0..8
    int K, N;
    chain_dims(p.d, i, K, N);
    const T *Wt = reinterpret_cast<const T *>(p.wt[l]);
    const float *bias = p.b[l];
    T *gout = reinterpret_cast<T *>(p.act[i + 1]);
    for (int t = wave; t < N / 32; t += 4) {
      f32x16_t acc;
      tile_mm<T>(xin, ldx, Wt, K, 32 * t, acc);
      const int col = 32 * t + (lane & 31);
      const float bb = bias[col];
      T tv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = acc_row(r, lane);
        float v = acc[r] + bb;
        v = v > 0.f ? v : 0.f;
        DT<T>::st(&tv[r], v);
        xout[row * ldx + col] = tv[r];
        gout[(int64_t)(r0 + row) * N + col] = tv[r];
      }
      if (i == 5 && p.act6t) {  // D3^T [d][R]: registers 4g..4g+3 = 4 consecutive rows
        T *dt = reinterpret_cast<T *>(p.act6t) + (int64_t)col * p.R + r0 + 4 * (lane >> 5);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if constexpr (sizeof(T) == 2)
            *reinterpret_cast<uint2 *>(dt + 8 * g) = *reinterpret_cast<const uint2 *>(&tv[4 * g]);
          else
            *reinterpret_cast<uint4 *>(dt + 8 * g) = *reinterpret_cast<const uint4 *>(&tv[4 * g]);
        }
      }
    }
    __syncthreads();
    T *tmp = xin;
    xin = xout;
    xout = tmp;
  }
}

// dX chain: one block per 32 rows carries dPre from d3 down to e1; every layer's dPre is written
// to global (gact) for the dW kernel.  H (the layer input) is needed only as the ReLU mask.
template <typename T>
__global__ __launch_bounds__(NT) void tower_bwd_chain_kernel(TowerP p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int MAXT = 8;  // dX tiles per wave (K <= 1024)
  const int ldx = p.maxw + 16 / (int)sizeof(T);
  T *Gr = reinterpret_cast<T *>(smem);
  T *Hr = Gr + RB * ldx;
  const int blk = blockIdx.x, r0 = blk * RB;
  const bool reg = r0 >= p.B;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  load_block<T>(reinterpret_cast<const T *>(p.gD3), p.d, r0, Gr, ldx, (T *)nullptr, 0);
  for (int i = 5; i >= 0; --i) {
    const int l = i < 3 ? i : i + (reg ? 3 : 0);
    int K, N;
    chain_dims(p.d, i, K, N);
    // layer input H (only its ReLU mask is needed): coalesced block copy into LDS
    load_block<T>(reinterpret_cast<const T *>(p.act[i]), K, r0, Hr, ldx, (T *)nullptr, 0);
    __syncthreads();
    const T *W = reinterpret_cast<const T *>(p.w[l]);    // [K][N]: row k is k-contiguous over N
    f32x16_t accs[MAXT];
#pragma unroll
    for (int q = 0; q < MAXT; ++q) {
      const int t = wave + 4 * q;
      if (t < K / 32) tile_mm<T>(Gr, ldx, W, N, 32 * t, accs[q]);
    }
    __syncthreads();  // every wave has finished reading Gr
    T *gout = i > 0 ? reinterpret_cast<T *>(p.gact[i - 1]) : nullptr;
#pragma unroll
    for (int q = 0; q < MAXT; ++q) {
      const int t = wave + 4 * q;
      if (t >= K / 32) continue;
      const int col = 32 * t + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = acc_row(r, lane);
        const int64_t go = (int64_t)(r0 + row) * K + col;
        const float h = DT<T>::ld(&Hr[row * ldx + col]);
        const float v = h > 0.f ? accs[q][r] : 0.f;
        if (i == 0) {
          p.gpre1[go] = v;
          if constexpr (sizeof(T) == 2) {
            if (p.gpre1t)
              reinterpret_cast<bf16_t *>(p.gpre1t)[(int64_t)col * ((p.R + 63) & ~63) + r0 + row] = f2bf(v);
          }
        } else {
          T tv;
          DT<T>::st(&tv, v);
          Gr[row * ldx + col] = tv;
          gout[go] = tv;
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ bf16 fast path (d <= 256)
// (templated on d: every layer's widths are compile-time constants, so no fragment load or MFMA
// sits behind a branch — a conditional load makes the compiler drain vmcnt before it)
// Same math as the kernels above, shaped for latency: 8 waves, one 32-column output tile per
// wave per layer, and the NEXT layer's weight fragments are loaded into registers while the
// current layer's MFMAs run — weights do not depend on the activations, so every layer after
// the first starts with its operands already in flight.
constexpr int FNT = 512;  // 8 waves
#ifndef TF_CPB   // cc_tower_bwd_chain_noise: cubes of F per 512-thread workgroup (2 or 4)
#define TF_CPB 4
#endif
constexpr int FB = 16;    // fragments per tile: reduction length <= 256

struct Frags {
  bf16x8_t f[FB];
};
// B fragments of the 32-column tile n0 of a [rows][K] k-contiguous matrix (rows = output cols)
__device__ __forceinline__ void issue_frags(Frags &F, const bf16_t *__restrict__ W, int K, int n0) {
  const int lane = threadIdx.x & 63;
  const bf16_t *row = W + (int64_t)(n0 + (lane & 31)) * K + 8 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < FB; ++j)
    if (16 * j < K) F.f[j] = *reinterpret_cast<const bf16x8_t *>(row + 16 * j);
}
// the same fragments from a fragment-packed image (cc_tower_args.wpf / wpb): fragment (t, j) is
// 64 lanes x 16 B contiguous, so each wave load reads 8 whole cache lines (the row-strided form
// touches 32 lines per load and refetches each line once per 16-k step)
__device__ __forceinline__ void issue_frags_packed(Frags &F, const bf16_t *__restrict__ P, int red, int t) {
  const int lane = threadIdx.x & 63;
  const bf16_t *base = P + ((int64_t)t * (red / 16) * 64 + lane) * 8;
#pragma unroll
  for (int j = 0; j < FB; ++j)
    if (16 * j < red) F.f[j] = *reinterpret_cast<const bf16x8_t *>(base + j * 512);
}
// packed-image element offset of fragment (t, j), lane, element e
__device__ __forceinline__ int64_t pack_off(int t, int j, int lane, int red) {
  return (((int64_t)t * (red / 16) + j) * 64 + lane) * 8;
}

// 32 rows x W (bf16, W <= 256) of a [R][W] activation into registers: issue now, store to LDS later
typedef __attribute__((ext_vector_type(4))) uint32_t u32v4;  // staging registers (HIP's uint4
                                                              // struct would be spilled to scratch)
struct RowRegs {
  u32v4 v[2];
};
__device__ __forceinline__ void rows_issue(RowRegs &Rg, const bf16_t *__restrict__ g, int W, int r0) {
  const int per = W / 8, nv = RB * per;
  const u32v4 *src = reinterpret_cast<const u32v4 *>(g + (int64_t)r0 * W);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = (int)threadIdx.x + u * FNT;
    if (i < nv) Rg.v[u] = src[i];
  }
}
__device__ __forceinline__ void rows_store(const RowRegs &Rg, int W, bf16_t *Xr, int ldx) {
  const int per = W / 8, nv = RB * per;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = (int)threadIdx.x + u * FNT;
    if (i < nv) *reinterpret_cast<u32v4 *>(Xr + (i / per) * ldx + (i % per) * 8) = Rg.v[u];
  }
}

__device__ __forceinline__ void consume_frags(const Frags &F, const bf16_t *A, int lda, int K,
                                              f32x16_t &acc) {
  const int lane = threadIdx.x & 63;
  const bf16_t *arow = A + (lane & 31) * lda + 8 * (lane >> 5);
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int j = 0; j < FB; ++j)
    if (16 * j < K)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8_t *>(arow + 16 * j),
                                                    F.f[j], acc, 0, 0, 0);
}

// Transposed product: with the packed B fragments as the MFMA's A operand and the LDS activation
// rows as its B operand the accumulators hold C^T — lane l owns batch row (l & 31) and columns
// (r & 3) + 8 (r >> 2) + 4 (l >> 5) of the tile, i.e. four runs of 4 consecutive columns — so the
// epilogue writes 8-B runs instead of 2-B scatters.  Same loads, same products.
__device__ __forceinline__ void consume_frags_t(const Frags &F, const bf16_t *A, int lda, int K,
                                                f32x16_t &acc) {
  const int lane = threadIdx.x & 63;
  const bf16_t *arow = A + (lane & 31) * lda + 8 * (lane >> 5);
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int j = 0; j < FB; ++j)
    if (16 * j < K)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F.f[j], *reinterpret_cast<const bf16x8_t *>(arow + 16 * j),
                                                    acc, 0, 0, 0);
}

__device__ __forceinline__ uint2 pack4_bf16(float a, float b, float c, float d) {
  return make_uint2((uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16), (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16));
}

// the block's 32 rows of an LDS image (pitch ldx) -> global [R][W] rows r0.., 16-B coalesced
__device__ __forceinline__ void rows_copy_out(const bf16_t *X, int ldx, bf16_t *__restrict__ g, int W, int r0) {
  const int per = W / 8, nv = RB * per;
  for (int i = threadIdx.x; i < nv; i += FNT) {
    const int row = i / per, c = (i % per) * 8;
    *reinterpret_cast<uint4 *>(g + (int64_t)(r0 + row) * W + c) = *reinterpret_cast<const uint4 *>(X + row * ldx + c);
  }
}
// ... transposed: dst [W][ld] (column c holds the block's rows r0..r0+31 contiguously), 16-B stores
__device__ __forceinline__ void cols_copy_out(const bf16_t *X, int ldx, bf16_t *__restrict__ dt, int W, int ld, int r0) {
  for (int i = threadIdx.x; i < W * 4; i += FNT) {
    const int c = i >> 2, q = i & 3;
    uint32_t w4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w4[e] = (uint32_t)X[(8 * q + 2 * e) * ldx + c] | ((uint32_t)X[(8 * q + 2 * e + 1) * ldx + c] << 16);
    *reinterpret_cast<uint4 *>(dt + (int64_t)c * ld + r0 + 8 * q) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}

// ... packed transposed (rows = the W features, reduction = batch rows): the block's rows are
// reduction steps j = r0/16, r0/16 + 1 of fragment columns t = 0 .. W/32-1 (the MFMA operand
// layout of the dW products, 1 KB per fragment)
__device__ __forceinline__ void pt_copy_out(const bf16_t *X, int ldx, bf16_t *__restrict__ dst, int W, int R, int r0) {
  for (int v = threadIdx.x; v < (W / 32) * 2 * 64; v += FNT) {
    const int ln = v & 63, jj = (v >> 6) & 1, tt = v >> 7;
    const bf16_t *src = X + (16 * jj + 8 * (ln >> 5)) * ldx + 32 * tt + (ln & 31);
    uint32_t w4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) w4[e] = (uint32_t)src[(2 * e) * ldx] | ((uint32_t)src[(2 * e + 1) * ldx] << 16);
    *reinterpret_cast<u32v4 *>(dst + pack_off(tt, r0 / 16 + jj, ln, R)) = u32v4{w4[0], w4[1], w4[2], w4[3]};
  }
}

constexpr int BIAS_MAX = 256 + 128 + 64 + 128 + 256 + 256;  // the six chain layers' widths, d <= 256
// offset of chain layer i's bias in the block's LDS bias image (widths 256, 128, 64, 128, 256, d)
__device__ __forceinline__ int bias_off(int i) {
  return i <= 0 ? 0 : i == 1 ? 256 : i == 2 ? 384 : i == 3 ? 448 : i == 4 ? 576 : 832;
}

// Workgroup barrier over LDS only: the chains hand only LDS images between their waves, and
// __syncthreads' release fence would also drain every outstanding global access (the next
// layer's prefetched weight fragments, the copy-out stores) at each layer boundary.
__device__ __forceinline__ void fast_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The fused D1 kernel's target-mask image (cc_tower_args.y_img, decout.hip): word column gw of the
// y row bitmasks, rows in the order the MFMA accumulator registers hold them — within every 32-row
// block, dword 2r + h = row (r & 3) + 8 (r >> 2) + 4h — so the 16 lane masks of one accumulator
// tile are 128 contiguous bytes (two scalar 64-B loads).  One block per (32-row block, 64 word
// columns): coalesced 256-B row reads into LDS, coalesced 128-B column writes.
constexpr int YI_W = 64;
__host__ __device__ inline int yimg_blocks(int B, int VW) { return (B / 32) * ((VW + YI_W - 1) / YI_W); }
__device__ __forceinline__ void yimg_block(const uint32_t *__restrict__ yb, int VW, int B, uint32_t *__restrict__ yimg,
                                           int tb) {
  extern __shared__ uint32_t ysm[];   // [32][YI_W + 1] (the launch's dynamic LDS)
  const int nrb = B / 32, rb = tb % nrb, w0 = (tb / nrb) * YI_W;
  for (int i = threadIdx.x; i < 32 * YI_W; i += blockDim.x) {
    const int row = i / YI_W, c = i % YI_W;
    ysm[row * (YI_W + 1) + c] = w0 + c < VW ? yb[(int64_t)(rb * 32 + row) * VW + w0 + c] : 0u;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < 32 * YI_W; o += blockDim.x) {
    const int j = o / 32, pos = o % 32;
    const int row = 8 * (pos >> 3) + 4 * (pos & 1) + ((pos >> 1) & 3);
    if (w0 + j < VW) yimg[(int64_t)(w0 + j) * B + rb * 32 + pos] = ysm[row * (YI_W + 1) + j];
  }
}

// blocks [R/RB, R/RB + nxt): the xt transposes; then the target-mask image's blocks
template <int D>
__global__ __launch_bounds__(FNT) void tower_fwd_fast_kernel(TowerP p, int nxt) {
  if ((int)blockIdx.x >= p.R / RB + nxt) {  // then the target-mask image
    yimg_block(p.yb, p.y_VW, p.B, p.yimg, (int)blockIdx.x - p.R / RB - nxt);
    return;
  }
  if ((int)blockIdx.x >= p.R / RB) {  // blocks past the chains: the xt transpose on the idle CUs
    xt_transpose_block(p.xb, p.xt_V, p.xt, p.xt_rows, (int)blockIdx.x - p.R / RB);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ __attribute__((aligned(16))) float bsm[BIAS_MAX];
  const int ldx = p.maxw + 8;
  bf16_t *X0 = reinterpret_cast<bf16_t *>(smem);
  bf16_t *X1 = X0 + RB * ldx;
  const int r0 = blockIdx.x * RB;
  const bool reg = r0 >= p.B;
  const int t = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5;
  const int nbias = bias_off(5) + D;
  Frags fr[2];
  TOWER_PROBE(0);
  // the block's input rows first (they gate the first MFMA), then the biases, then the weights
  RowRegs rg;
  rows_issue(rg, reinterpret_cast<const bf16_t *>(p.act[0]), D, r0);
  float bv[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int c = (int)threadIdx.x + q * FNT;
    bv[q] = 0.f;
    if (c < nbias) {
      const int i = c < 256 ? 0 : c < 384 ? 1 : c < 448 ? 2 : c < 576 ? 3 : c < 832 ? 4 : 5;
      const int l = i < 3 ? i : i + (reg ? 3 : 0);
      bv[q] = p.b[l][c - bias_off(i)];
    }
  }
  auto issue = [&](int i, int slot) {
    const int l = i < 3 ? i : i + (reg ? 3 : 0);
    int K, N;
    chain_dims(D, i, K, N);
    if (t < N / 32) {
      if (p.packed)
        issue_frags_packed(fr[slot], p.wpf[l], K, t);
      else
        issue_frags(fr[slot], reinterpret_cast<const bf16_t *>(p.wt[l]), K, 32 * t);
    }
  };
  issue(0, 0);
  rows_store(rg, D, X0, ldx);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int c = (int)threadIdx.x + q * FNT;
    if (c < nbias) bsm[c] = bv[q];
  }
  fast_barrier();
  TOWER_PROBE(1);
  bf16_t *xin = X0, *xout = X1;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    int K, N;
    chain_dims(D, i, K, N);
    if (i < 5) issue(i + 1, (i + 1) & 1);  // next layer's weights fly during this layer
    f32x16_t acc;
    if (t < N / 32) consume_frags_t(fr[i & 1], xin, ldx, K, acc);
    TOWER_PROBE(2 + 3 * i);
    // the previous layer's output (this layer's input, read-only now) to global while the MFMAs
    // run: rows for the backward's ReLU masks, packed transposed for the dW kernel
    if (i > 0) rows_copy_out(xin, ldx, reinterpret_cast<bf16_t *>(p.act[i]), K, r0);
    if (p.dwpacked) pt_copy_out(xin, ldx, p.hpt[i], K, p.R, r0);
    if (t < N / 32) {
      const int row = lane & 31, cb = 32 * t + 4 * half;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b4 = *reinterpret_cast<const float4 *>(bsm + bias_off(i) + cb + 8 * g);
        *reinterpret_cast<uint2 *>(xout + row * ldx + cb + 8 * g) =
            pack4_bf16(fmaxf(acc[4 * g] + b4.x, 0.f), fmaxf(acc[4 * g + 1] + b4.y, 0.f),
                       fmaxf(acc[4 * g + 2] + b4.z, 0.f), fmaxf(acc[4 * g + 3] + b4.w, 0.f));
      }
      TOWER_PROBE(3 + 3 * i);
    }
    fast_barrier();
    TOWER_PROBE(4 + 3 * i);
    bf16_t *tmp = xin;
    xin = xout;
    xout = tmp;
  }
  // D3 (the last layer's output): rows, D3^T [d][R], and the packed operand images of the fused
  // output-layer kernel
  const int dd = D;
  rows_copy_out(xin, ldx, reinterpret_cast<bf16_t *>(p.act[6]), dd, r0);
  if (p.act6t) cols_copy_out(xin, ldx, reinterpret_cast<bf16_t *>(p.act6t), dd, p.R, r0);
  if (p.act6p) {  // D3 as the logits' A operand: fragments (blockIdx.x, j)
    for (int v = threadIdx.x; v < (dd / 16) * 64; v += FNT) {
      const int j = v >> 6, ln = v & 63;
      *reinterpret_cast<u32v4 *>(p.act6p + pack_off(blockIdx.x, j, ln, dd)) =
          *reinterpret_cast<const u32v4 *>(xin + (ln & 31) * ldx + 16 * j + 8 * (ln >> 5));
    }
  }
  if (p.act6tp) pt_copy_out(xin, ldx, p.act6tp, dd, p.R, r0);  // D3^T: the dWo A operand
}

// ADAM: blocks past the chains run TF Adam over a flat range (cc_tower_bwd_chain_adam) on the CUs
// the 16-32 latency-bound chain blocks leave idle; the chains launch first, so they start at once.
// NOISE (cc_tower_bwd_chain_noise): the next blocks draw F of the NEXT step, one cube per block on
// all 512 threads (noise_dev.hpp) — F is latency-bound like the chains, and by the tower backward
// every batch buffer F writes (x rows / bits, y bits, reg rows) has been read for this step.
template <int D, bool ADAM, bool NOISE = false>
__global__ __launch_bounds__(FNT) void tower_bwd_chain_fast_kernel(TowerP p, cc_adam::Args ad,
                                                                   cc_adam::Args ad1, const int64_t *ad_state,
                                                                   cc_noise_args na = {}, int64_t bpe = 1) {
  // F: TF_CPB cubes per block, one per FNT / TF_CPB threads (the chains' 173 VGPRs allow one
  // 512-thread block per CU: a cube per block would need two rounds of the ~240 free CUs)
  constexpr int FT = FNT / TF_CPB;
  const int nchain = p.R / RB, nf = NOISE ? (na.B + TF_CPB - 1) / TF_CPB : 0;
  if (NOISE && (int)blockIdx.x >= nchain && (int)blockIdx.x < nchain + nf) {
    extern __shared__ __attribute__((aligned(16))) uint32_t fsm[];
    __shared__ int s_k[TF_CPB];
    const int64_t step = na.state[0];
    int64_t batch = na.state[1] + 1, epoch = na.state[2];
    if (batch >= bpe) {
      batch = 0;
      epoch += 1;
    }
    const int h = threadIdx.x / FT, cube = TF_CPB * ((int)blockIdx.x - nchain) + h;
    const int fw = 4 * ((na.V + 31) / 32) + FT + 1;   // one slice's LDS words
    // (the last block's slices past B end here: their waves leave the barriers to the others)
    if (cube < na.B) ccnoise::noise_block<FT>(na, fsm + h * fw, s_k[h], cube, step + 1, batch, epoch);
    return;
  }
  if (ADAM && (int)blockIdx.x >= nchain + nf) {  // (two flat ranges, one after the other)
    const int b = (int)blockIdx.x - nchain - nf, nb = (int)gridDim.x - nchain - nf;
    cc_adam::range_u<4>(ad, ad_state[0], b, nb);
    if (ad1.n > 0) cc_adam::range_u<4>(ad1, ad_state[0], b, nb);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ldx = p.maxw + 8;
  bf16_t *Gr = reinterpret_cast<bf16_t *>(smem);
  const int r0 = blockIdx.x * RB;
  const bool reg = r0 >= p.B;
  const int t = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5;
  const int row = lane & 31, cb = 32 * t + 4 * half;
  Frags fr[2];
  auto issue_layer = [&](int i, int slot) {
    const int l = i < 3 ? i : i + (reg ? 3 : 0);
    int K, N;
    chain_dims(D, i, K, N);
    if (t < K / 32) {
      if (p.packed)
        issue_frags_packed(fr[slot], p.wpb[l], N, t);
      else
        issue_frags(fr[slot], reinterpret_cast<const bf16_t *>(p.w[l]), N, 32 * t);
    }
  };
  RowRegs rg;
  rows_issue(rg, reinterpret_cast<const bf16_t *>(p.gD3), D, r0);
  issue_layer(5, 1);
  rows_store(rg, D, Gr, ldx);
  fast_barrier();
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    int K, N;
    chain_dims(D, i, K, N);
    if (i > 0) issue_layer(i - 1, (i - 1) & 1);
    // the layer input's ReLU mask at this lane's accumulator positions: lands during the MFMAs
    uint2 hm[4];
    if (t < K / 32) {
      const bf16_t *H = reinterpret_cast<const bf16_t *>(p.act[i]) + (int64_t)(r0 + row) * K + cb;
#pragma unroll
      for (int g = 0; g < 4; ++g) hm[g] = *reinterpret_cast<const uint2 *>(H + 8 * g);
    }
    f32x16_t acc;
    if (t < K / 32) consume_frags_t(fr[i & 1], Gr, ldx, N, acc);
    // this layer's incoming gradient G_i (Gr, read-only until the barrier) to global while the
    // MFMAs run: rows (the dW fallback) and packed transposed for the dW kernel
    if (i < 5) rows_copy_out(Gr, ldx, reinterpret_cast<bf16_t *>(p.gact[i]), N, r0);
    if (p.dwpacked) pt_copy_out(Gr, ldx, p.gpt[i], N, p.R, r0);
    fast_barrier();  // every wave has finished reading Gr
    if (t < K / 32) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float v0 = __uint_as_float(hm[g].x << 16) > 0.f ? acc[4 * g] : 0.f;
        const float v1 = __uint_as_float(hm[g].x & 0xFFFF0000u) > 0.f ? acc[4 * g + 1] : 0.f;
        const float v2 = __uint_as_float(hm[g].y << 16) > 0.f ? acc[4 * g + 2] : 0.f;
        const float v3 = __uint_as_float(hm[g].y & 0xFFFF0000u) > 0.f ? acc[4 * g + 3] : 0.f;
        if (i == 0)
          *reinterpret_cast<float4 *>(p.gpre1 + (int64_t)(r0 + row) * K + cb + 8 * g) = make_float4(v0, v1, v2, v3);
        *reinterpret_cast<uint2 *>(Gr + row * ldx + cb + 8 * g) = pack4_bf16(v0, v1, v2, v3);
      }
    }
    fast_barrier();
    // (G_{i-1} for i > 0 is copied out during the next layer's MFMAs)
    if (i == 0 && p.gpre1p)  // dPre1 as packed transposed fragments (reduction ceil64(R)): cc_embed_grad_packed
      pt_copy_out(Gr, ldx, p.gpre1p, K, (p.R + 63) & ~63, r0);
    else if (i == 0 && p.gpre1t)  // dPre1^T [d][ceil64(R)] (bf16) for cc_embed_grad_mfma
      cols_copy_out(Gr, ldx, reinterpret_cast<bf16_t *>(p.gpre1t), K, (p.R + 63) & ~63, r0);
  }
}

// ------------------------------------------------------------------ bf16 wide path (256 < d <= 1024)
// The d <= 256 kernels above give each wave ONE 32-column tile per layer with its whole reduction
// (<= 256 = 16 fragments) in registers.  At d = 1024 (config 5) the first / last layers have 32
// output tiles or a 1,024-long reduction, so a wave's work becomes a stream of items (layer, tile,
// 256-long reduction chunk) in layer order: the next item's fragments (possibly of a later layer)
// load while the current item's MFMAs run, and a wave crossing a layer boundary joins that
// layer's barrier first — every wave passes every barrier once, in order, whatever its items.
// Activations ping-pong between two LDS images (forward: layer in / out; backward: G in / dH out)
// so a tile's epilogue never waits for the other waves' reads.
constexpr int WBIAS_MAX = 832 + 1024;  // bias_off(5) + d


// a[k] of a kernel-argument pointer array with a runtime layer index, as a select chain over
// constant-offset reads: indexing the array directly compiles to a global load whose vmcnt wait
// (in-order counter) drained the in-flight fragments before every item
template <typename T, int N>
__device__ __forceinline__ T pick(const T (&a)[N], int k) {
  T r = a[0];
#pragma unroll
  for (int j = 1; j < N; ++j) r = k == j ? a[j] : r;
  return r;
}

struct WItem {
  int i, t, c, nch, red;  // chain layer, 32-column tile, reduction chunk, chunks per tile, reduction
};
// the q-th item of wave w (forward: layers 0..5, tiles of N, reduction K; backward: layers 5..0,
// tiles of K, reduction N)
__device__ __forceinline__ bool witem(int d, bool fwd, int w, int q, WItem &it) {
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int i = fwd ? s : 5 - s;
    int K, N;
    chain_dims(d, i, K, N);
    const int nt = (fwd ? N : K) >> 5, red = fwd ? K : N;
    const int nch = (red + 255) >> 8;
    const int mine = nt > w ? (nt - w + 7) >> 3 : 0;
    const int cnt = mine * nch;
    if (q < cnt) {
      it.i = i;
      it.t = w + 8 * (q / nch);
      it.c = q % nch;
      it.nch = nch;
      it.red = red;
      return true;
    }
    q -= cnt;
  }
  return false;
}
// fragments j = 16c .. 16c + 15 of tile t of a packed image with reduction `red`.  Always 16
// unconditional loads (a chunk shorter than 16 fragments re-reads its last one: same lines, L1
// hits): a conditional load compiles to a branch, and the compiler then drains vmcnt to zero
// before it — which serialises the item pipeline (the first d = 1024 forward ran 50 us that way)
__device__ __forceinline__ void issue_chunk(Frags &F, const bf16_t *__restrict__ P, const WItem &it) {
  const int lane = threadIdx.x & 63;
  const bf16_t *base = P + (((int64_t)it.t * (it.red / 16) + 16 * it.c) * 64 + lane) * 8;
  const int last = min(FB, it.red / 16 - 16 * it.c) - 1;
#pragma unroll
  for (int j = 0; j < FB; ++j) F.f[j] = *reinterpret_cast<const bf16x8_t *>(base + min(j, last) * 512);
}
template <int NF>
__device__ __forceinline__ void mfma_chunk(const Frags &F, const bf16_t *arow, f32x16_t &acc) {
#pragma unroll
  for (int j = 0; j < NF; ++j)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F.f[j], *reinterpret_cast<const bf16x8_t *>(arow + 16 * j), acc,
                                                  0, 0, 0);
}
// acc (+)= chunk c of the transposed product (packed weights = A, LDS rows = B; see consume_frags_t).
// A chunk holds 16, 12, 8 or 4 fragments (reductions are multiples of 64): static MFMA counts.
__device__ __forceinline__ void consume_chunk_t(const Frags &F, const bf16_t *A, int lda, const WItem &it,
                                                f32x16_t &acc) {
  const int lane = threadIdx.x & 63;
  const bf16_t *arow = A + (lane & 31) * lda + 8 * (lane >> 5) + 256 * it.c;
  if (it.c == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  }
  const int nf = min(FB, it.red / 16 - 16 * it.c);
  if (nf == 16)
    mfma_chunk<16>(F, arow, acc);
  else if (nf == 12)
    mfma_chunk<12>(F, arow, acc);
  else if (nf == 8)
    mfma_chunk<8>(F, arow, acc);
  else
    mfma_chunk<4>(F, arow, acc);
}

__global__ __launch_bounds__(FNT) void tower_fwd_wide_kernel(TowerP p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ __attribute__((aligned(16))) float bsm[WBIAS_MAX];
  const int ldx = p.maxw + 8;
  bf16_t *xin = reinterpret_cast<bf16_t *>(smem);
  bf16_t *xout = xin + RB * ldx;
  const int r0 = blockIdx.x * RB;
  const bool reg = r0 >= p.B;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, half = lane >> 5;
  const int d = p.d, nbias = bias_off(5) + d;
  auto wimg = [&](int i) { return pick(p.wpf, i < 3 ? i : i + (reg ? 3 : 0)); };
  Frags fr[2];
  WItem a, b;
  bool ha = witem(d, true, w, 0, a);
  if (ha) issue_chunk(fr[0], wimg(a.i), a);
  for (int c = threadIdx.x; c < nbias; c += FNT) {
    const int i = c < 256 ? 0 : c < 384 ? 1 : c < 448 ? 2 : c < 576 ? 3 : c < 832 ? 4 : 5;
    const int l = i < 3 ? i : i + (reg ? 3 : 0);
    bsm[c] = p.b[l][c - bias_off(i)];
  }
  load_block_n<bf16_t, FNT>(reinterpret_cast<const bf16_t *>(p.act[0]), d, r0, xin, ldx);
  fast_barrier();
  int layer = 0;
  auto layer_start = [&](int i) {  // the layer's input (read-only now) to global: rows + packed transposed
    int K, N;
    chain_dims(d, i, K, N);
    if (i > 0) rows_copy_out(xin, ldx, reinterpret_cast<bf16_t *>(pick(p.act, i)), K, r0);
    if (p.dwpacked) pt_copy_out(xin, ldx, pick(p.hpt, i), K, p.R, r0);
  };
  auto advance = [&]() {
    fast_barrier();
    bf16_t *tmp = xin;
    xin = xout;
    xout = tmp;
    if (++layer < 6) layer_start(layer);
  };
  layer_start(0);
  f32x16_t acc;
  auto step = [&](const Frags &F, const WItem &it) {
    while (layer < it.i) advance();
    consume_chunk_t(F, xin, ldx, it, acc);
    if (it.c == it.nch - 1) {
      const int row = lane & 31, cb = 32 * it.t + 4 * half;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b4 = *reinterpret_cast<const float4 *>(bsm + bias_off(it.i) + cb + 8 * g);
        *reinterpret_cast<uint2 *>(xout + row * ldx + cb + 8 * g) =
            pack4_bf16(fmaxf(acc[4 * g] + b4.x, 0.f), fmaxf(acc[4 * g + 1] + b4.y, 0.f),
                       fmaxf(acc[4 * g + 2] + b4.z, 0.f), fmaxf(acc[4 * g + 3] + b4.w, 0.f));
      }
    }
  };
  int q = 0;
  while (ha) {
    const bool hb = witem(d, true, w, q + 1, b);
    if (hb) issue_chunk(fr[1], wimg(b.i), b);
    step(fr[0], a);
    if (!hb) break;
    ha = witem(d, true, w, q + 2, a);
    if (ha) issue_chunk(fr[0], wimg(a.i), a);
    step(fr[1], b);
    q += 2;
  }
  while (layer < 6) advance();
  // D3 = the last layer's output (now xin): rows and D3^T [d][R], and the packed operand images
  // of the fused output-layer kernels (d = 512: cc_dec_bce_dw)
  rows_copy_out(xin, ldx, reinterpret_cast<bf16_t *>(p.act[6]), d, r0);
  if (p.act6t) cols_copy_out(xin, ldx, reinterpret_cast<bf16_t *>(p.act6t), d, p.R, r0);
  if (p.act6p) {  // D3 as the logits' A operand: fragments (blockIdx.x, j)
    for (int v = threadIdx.x; v < (d / 16) * 64; v += FNT) {
      const int j = v >> 6, ln = v & 63;
      *reinterpret_cast<u32v4 *>(p.act6p + pack_off(blockIdx.x, j, ln, d)) =
          *reinterpret_cast<const u32v4 *>(xin + (ln & 31) * ldx + 16 * j + 8 * (ln >> 5));
    }
  }
  if (p.act6tp) pt_copy_out(xin, ldx, p.act6tp, d, p.R, r0);  // D3^T: the dWo A operand
  if (p.d3q) {  // config 5: D3's MX-FP8 images (cc_quant_mx8's layout and rule, from the LDS copy)
    const int nbr = d / 32;
    for (int t = threadIdx.x; t < RB * nbr; t += FNT) {  // rows image: K = d, block b of row r
      const int r = t / nbr, b = t % nbr;
      float v[32];
      float amax = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32v4 u = *reinterpret_cast<const u32v4 *>(xin + r * ldx + 32 * b + 8 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[8 * q + 2 * e] = __uint_as_float(u[e] << 16);
          v[8 * q + 2 * e + 1] = __uint_as_float(u[e] & 0xFFFF0000u);
        }
      }
#pragma unroll
      for (int e = 0; e < 32; ++e) amax = fmaxf(amax, fabsf(v[e]));
      const int ex = cc_mx8::block_exp(amax);
      uint32_t w[8];
      cc_mx8::encode32(v, ex, w);
      uint4 *dst = reinterpret_cast<uint4 *>(p.d3q + (int64_t)(r0 + r) * d + 32 * b);
      dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
      dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
      p.d3qs[(int64_t)(r0 + r) * nbr + b] = (uint8_t)(ex + 127);
    }
    for (int c = threadIdx.x; c < d; c += FNT) {  // transposed image: K = rows, the block's 32 rows
      float v[32];
      float amax = 0.f;
#pragma unroll
      for (int r = 0; r < 32; ++r) {
        v[r] = __uint_as_float((uint32_t)reinterpret_cast<const uint16_t *>(xin)[r * ldx + c] << 16);
        amax = fmaxf(amax, fabsf(v[r]));
      }
      const int ex = cc_mx8::block_exp(amax);
      uint32_t w[8];
      cc_mx8::encode32(v, ex, w);
      uint4 *dst = reinterpret_cast<uint4 *>(p.d3tq + (int64_t)c * p.R + r0);
      dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
      dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
      p.d3tqs[(int64_t)c * (p.R / 32) + r0 / 32] = (uint8_t)(ex + 127);
    }
  }
}

__global__ __launch_bounds__(FNT) void tower_bwd_chain_wide_kernel(TowerP p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ldx = p.maxw + 8;
  bf16_t *gin = reinterpret_cast<bf16_t *>(smem);
  bf16_t *gout = gin + RB * ldx;
  const int r0 = blockIdx.x * RB;
  const bool reg = r0 >= p.B;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, half = lane >> 5;
  const int row = lane & 31;
  const int d = p.d;
  auto wimg = [&](int i) { return pick(p.wpb, i < 3 ? i : i + (reg ? 3 : 0)); };
  Frags fr[2];
  WItem a, b;
  bool ha = witem(d, false, w, 0, a);
  if (ha) issue_chunk(fr[0], wimg(a.i), a);
  load_block_n<bf16_t, FNT>(reinterpret_cast<const bf16_t *>(p.gD3), d, r0, gin, ldx);
  fast_barrier();
  int layer = 5;  // the layer whose incoming gradient gin holds
  auto layer_start = [&](int i) {  // G_i (read-only now) to global: rows (the dW fallback) + packed
    int K, N;
    chain_dims(d, i, K, N);
    if (i < 5) rows_copy_out(gin, ldx, reinterpret_cast<bf16_t *>(pick(p.gact, i)), N, r0);
    if (p.dwpacked) pt_copy_out(gin, ldx, pick(p.gpt, i), N, p.R, r0);
  };
  auto advance = [&]() {
    fast_barrier();
    bf16_t *tmp = gin;
    gin = gout;
    gout = tmp;
    if (--layer >= 0) layer_start(layer);
  };
  layer_start(5);
  f32x16_t acc;
  uint2 hm[4];
  // the ReLU mask of item it's layer input at this lane's accumulator positions, loaded BEFORE
  // the next item's fragments are issued (vmcnt retires in order: the epilogue's wait for the
  // mask then leaves those fragments in flight); every chunk, no branch
  auto mask_load = [&](const WItem &it) {
    int K, N;
    chain_dims(d, it.i, K, N);
    const bf16_t *H = reinterpret_cast<const bf16_t *>(pick(p.act, it.i)) + (int64_t)(r0 + row) * K + 32 * it.t + 4 * half;
#pragma unroll
    for (int g = 0; g < 4; ++g) hm[g] = *reinterpret_cast<const uint2 *>(H + 8 * g);
  };
  auto step = [&](const Frags &F, const WItem &it) {
    while (layer > it.i) advance();
    int K, N;
    chain_dims(d, it.i, K, N);
    const int cb = 32 * it.t + 4 * half;
    consume_chunk_t(F, gin, ldx, it, acc);
    if (it.c == it.nch - 1) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float v0 = __uint_as_float(hm[g].x << 16) > 0.f ? acc[4 * g] : 0.f;
        const float v1 = __uint_as_float(hm[g].x & 0xFFFF0000u) > 0.f ? acc[4 * g + 1] : 0.f;
        const float v2 = __uint_as_float(hm[g].y << 16) > 0.f ? acc[4 * g + 2] : 0.f;
        const float v3 = __uint_as_float(hm[g].y & 0xFFFF0000u) > 0.f ? acc[4 * g + 3] : 0.f;
        if (it.i == 0)
          *reinterpret_cast<float4 *>(p.gpre1 + (int64_t)(r0 + row) * K + cb + 8 * g) = make_float4(v0, v1, v2, v3);
        *reinterpret_cast<uint2 *>(gout + row * ldx + cb + 8 * g) = pack4_bf16(v0, v1, v2, v3);
      }
    }
  };
  int q = 0;
  while (ha) {
    mask_load(a);
    const bool hb = witem(d, false, w, q + 1, b);
    if (hb) issue_chunk(fr[1], wimg(b.i), b);
    step(fr[0], a);
    if (!hb) break;
    mask_load(b);
    ha = witem(d, false, w, q + 2, a);
    if (ha) issue_chunk(fr[0], wimg(a.i), a);
    step(fr[1], b);
    q += 2;
  }
  while (layer >= 0) advance();
  // dPre1 (now gin) for the W1 gradient: packed transposed fragments or dPre1^T [d][ceil64(R)]
  if (p.gpre1p)
    pt_copy_out(gin, ldx, p.gpre1p, d, (p.R + 63) & ~63, r0);
  else if (p.gpre1t)
    cols_copy_out(gin, ldx, reinterpret_cast<bf16_t *>(p.gpre1t), d, (p.R + 63) & ~63, r0);
}

// dW partials: one block per (chain layer i, 32-row block): slab[blk][i] = H^T G over the block's
// rows (A = H^T, B = G from transposed LDS images, MFMA), db = colsum G.  Spreads the slab writes
// over 6x more CUs than the chain.
template <typename T>
__global__ __launch_bounds__(NT) void tower_dw_kernel(TowerP p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ldt = RB + 16 / (int)sizeof(T);
  T *Ht = reinterpret_cast<T *>(smem);
  T *Gt = Ht + p.maxw * ldt;
  const int nb = p.R / RB;
  const int i = blockIdx.x / nb, blk = blockIdx.x % nb, r0 = blk * RB;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5;
  int K, N;
  chain_dims(p.d, i, K, N);
  const T *H = reinterpret_cast<const T *>(p.act[i]);
  const T *G = reinterpret_cast<const T *>(i == 5 ? p.gD3 : p.gact[i]);
  load_block_t<T>(H, K, r0, Ht, ldt);
  load_block_t<T>(G, N, r0, Gt, ldt);
  __syncthreads();
  float *sw = p.slab + (int64_t)blk * p.slab_elems + slab_off(p.d, i);
  const int ntn = N / 32, nt = (K / 32) * ntn;
  for (int t = wave; t < nt; t += 4) {
    const int k0 = 32 * (t / ntn), n0 = 32 * (t % ntn);
    f32x16_t acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const T *arow = Ht + (k0 + (lane & 31)) * ldt;
    const T *brow = Gt + (n0 + (lane & 31)) * ldt;
#pragma unroll
    for (int kk = 0; kk < RB; kk += TMma<T>::KM)
      TMma<T>::mma(TMma<T>::ld(arow, kk, half), TMma<T>::ld(brow, kk, half), acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) sw[(int64_t)(k0 + acc_row(r, lane)) * N + n0 + (lane & 31)] = acc[r];
  }
  for (int n = threadIdx.x; n < N; n += NT) {
    float s = 0.f;
    const T *g = Gt + n * ldt;
    for (int b = 0; b < RB; ++b) s += DT<T>::ld(&g[b]);
    sw[(int64_t)K * N + n] = s;
  }
}

// grads[l] = sum over the blocks that touched layer l of their slab partials, in block order.
// Tower weight gradients without slabs (bf16 operands): one workgroup per 32 x 32 tile of one
// layer's dW = H^T G over all of that layer's rows (encoder: R rows; each decoder branch: its B
// rows).  The 4 waves split the rows; each stages its rows of H[:, k0:k0+32] and G[:, n0:n0+32]
// transposed in LDS ([col][row], 16-B MFMA fragment reads), accumulates with 32x32x16 MFMAs in
// row order, and the 4 partial tiles are added in wave order (deterministic).  Tiles of the
// first k-block also sum G's columns: the bias gradient.  Replaces tower_dw + tower_reduce.
constexpr int DW_NT = 256;

__device__ __forceinline__ bool dw_job(const TowerP &p, int bid, int &l, int &i, int &k0, int &n0,
                                       int &row0, int &nrows) {
  const int L = p.R > p.B ? 9 : 6;
  for (l = 0; l < L; ++l) {
    i = l < 6 ? l : l - 3;
    int K, N;
    chain_dims(p.d, i, K, N);
    const int tn = N / 32, nt = (K / 32) * tn;
    if (bid < nt) {
      k0 = 32 * (bid / tn);
      n0 = 32 * (bid % tn);
      row0 = l < 6 ? 0 : p.B;
      nrows = l < 3 ? p.R : (l < 6 ? p.B : p.R - p.B);   // reg branch: rows [B, R)
      return true;
    }
    bid -= nt;
  }
  return false;
}

__global__ __launch_bounds__(DW_NT) void tower_dw_tiled_kernel(TowerP p, int rpw) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int l, i, k0, n0, row0, nrows;
  if (!dw_job(p, blockIdx.x, l, i, k0, n0, row0, nrows)) return;
  int K, N;
  chain_dims(p.d, i, K, N);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5;
  const int ldr = rpw + 8;  // LDS row pitch (bf16): 16-B aligned, spreads the banks
  bf16_t *Ht = reinterpret_cast<bf16_t *>(smem) + (size_t)wave * 2 * 32 * ldr;
  bf16_t *Gt = Ht + 32 * ldr;
  const bf16_t *H = reinterpret_cast<const bf16_t *>(p.act[i]);
  const bf16_t *G = reinterpret_cast<const bf16_t *>(i == 5 ? p.gD3 : p.gact[i]);
  const int wr0 = wave * rpw;  // this wave's rows: [wr0, wr0 + rpw) of the layer's rows
  // stage: 4 lanes per row (8 bf16 = 16 B each), 16 rows per pass; rows past nrows are zeros
  for (int rr = lane >> 2; rr < rpw; rr += 16) {
    const int r = wr0 + rr, c8 = (lane & 3) * 8;
    uint4 hv = make_uint4(0u, 0u, 0u, 0u), gv = make_uint4(0u, 0u, 0u, 0u);
    if (r < nrows) {
      hv = *reinterpret_cast<const uint4 *>(H + (int64_t)(row0 + r) * K + k0 + c8);
      gv = *reinterpret_cast<const uint4 *>(G + (int64_t)(row0 + r) * N + n0 + c8);
    }
    const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w}, gw[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      Ht[(c8 + 2 * e) * ldr + rr] = (bf16_t)(hw[e] & 0xFFFFu);
      Ht[(c8 + 2 * e + 1) * ldr + rr] = (bf16_t)(hw[e] >> 16);
      Gt[(c8 + 2 * e) * ldr + rr] = (bf16_t)(gw[e] & 0xFFFFu);
      Gt[(c8 + 2 * e + 1) * ldr + rr] = (bf16_t)(gw[e] >> 16);
    }
  }
  __syncthreads();
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const bf16_t *arow = Ht + (lane & 31) * ldr;
  const bf16_t *brow = Gt + (lane & 31) * ldr;
  for (int kk = 0; kk < rpw; kk += 16)
    TMma<bf16_t>::mma(TMma<bf16_t>::ld(arow, kk, half), TMma<bf16_t>::ld(brow, kk, half), acc);
  float cs = 0.f;  // bias: this wave's rows of G column n0 + lane (lanes 0..31)
  if (k0 == 0 && lane < 32)
    for (int rr = 0; rr < rpw; ++rr) cs += bf2f(Gt[lane * ldr + rr]);
  __syncthreads();  // the staged operands are consumed: reuse the LDS for the partial tiles
  float *part = reinterpret_cast<float *>(smem);  // [4][32][33] + [4][32]
  float *pcs = part + 4 * 32 * 33;
#pragma unroll
  for (int r = 0; r < 16; ++r) part[(wave * 32 + acc_row(r, lane)) * 33 + (lane & 31)] = acc[r];
  if (lane < 32) pcs[wave * 32 + lane] = cs;
  __syncthreads();
  float *gw = p.gw[l];
  for (int e = threadIdx.x; e < 32 * 32; e += DW_NT) {
    const int kr = e >> 5, nc = e & 31;
    float v = part[(0 * 32 + kr) * 33 + nc];
#pragma unroll
    for (int w = 1; w < 4; ++w) v += part[(w * 32 + kr) * 33 + nc];
    gw[(int64_t)(k0 + kr) * N + n0 + nc] = v;
  }
  if (k0 == 0 && threadIdx.x < 32)
    p.gb[l][n0 + threadIdx.x] = pcs[threadIdx.x] + pcs[32 + threadIdx.x] + pcs[64 + threadIdx.x] +
                                pcs[96 + threadIdx.x];
}

// dW from the packed transposed images: one wave per 32x32 tile of one layer, dW[k0.., n0..] =
// sum over the layer's rows of H^T G as a chain of v_mfma_f32_32x32x16_bf16 whose A / B fragments
// are whole 1 KB runs of hpt / gpt (no LDS staging, no cross-wave reduce); db from the same B
// fragments on the k0 == 0 tiles.  Rows in order: deterministic.
constexpr int DWP_U = 8;  // fragment pairs in flight per lane
__global__ __launch_bounds__(64) void tower_dw_packed_kernel(TowerP p) {
  int l, i, k0, n0, row0, nrows;
  if (!dw_job(p, blockIdx.x, l, i, k0, n0, row0, nrows)) return;
  int K, N;
  chain_dims(p.d, i, K, N);
  const int lane = threadIdx.x, half = lane >> 5;
  const int R = p.R, j0 = row0 / 16, nj = nrows / 16;
  const bf16_t *ha = p.hpt[i] + pack_off(k0 / 32, j0, lane, R);
  const bf16_t *gb = p.gpt[i] + pack_off(n0 / 32, j0, lane, R);
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float cs = 0.f;
  const bool bias = k0 == 0;
  int j = 0;
  for (; j + DWP_U <= nj; j += DWP_U) {
    bf16x8_t a[DWP_U], b[DWP_U];
#pragma unroll
    for (int u = 0; u < DWP_U; ++u) {
      a[u] = *reinterpret_cast<const bf16x8_t *>(ha + (j + u) * 512);
      b[u] = *reinterpret_cast<const bf16x8_t *>(gb + (j + u) * 512);
    }
#pragma unroll
    for (int u = 0; u < DWP_U; ++u) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u], b[u], acc, 0, 0, 0);
      if (bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cs += (float)b[u][e];
      }
    }
  }
  for (; j < nj; ++j) {
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t *>(ha + j * 512);
    const bf16x8_t b = *reinterpret_cast<const bf16x8_t *>(gb + j * 512);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    if (bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) cs += (float)b[e];
    }
  }
  float *gw = p.gw[l] + (int64_t)(k0 + 4 * half) * N + n0 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) gw[(int64_t)((r & 3) + 8 * (r >> 2)) * N] = acc[r];
  if (bias) {
    cs += __shfl_xor(cs, 32);
    if (half == 0) p.gb[l][n0 + lane] = cs;
  }
}

// Row-split form for tall layers (full-mode regulariser: ~22k rows per chain): job (tile, split s)
// accumulates rows chunk s of the tile's chain into part[(job * S + s)] (the lane's 16 accumulators
// + its bias partial); tower_dw_split_reduce adds the S partials of each tile in split order
// (deterministic) — the one-wave-per-tile chain over 22k rows left most of the chip idle.
constexpr int DWS_STRIDE = 64 * 16 + 64;  // floats per (job, split) partial
__global__ __launch_bounds__(64) void tower_dw_packed_split_kernel(TowerP p, int S, float *__restrict__ part) {
  int l, i, k0, n0, row0, nrows;
  const int job = blockIdx.x, sp = blockIdx.y;
  if (!dw_job(p, job, l, i, k0, n0, row0, nrows)) return;
  const int lane = threadIdx.x;
  const int R = p.R, nj = nrows / 16, chunk = (nj + S - 1) / S;
  const int ja = min(nj, sp * chunk), jb = min(nj, ja + chunk);
  const int j0 = row0 / 16;
  const bf16_t *ha = p.hpt[i] + pack_off(k0 / 32, j0, lane, R);
  const bf16_t *gb = p.gpt[i] + pack_off(n0 / 32, j0, lane, R);
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float cs = 0.f;
  const bool bias = k0 == 0;
  int j = ja;
  for (; j + DWP_U <= jb; j += DWP_U) {
    bf16x8_t a[DWP_U], b[DWP_U];
#pragma unroll
    for (int u = 0; u < DWP_U; ++u) {
      a[u] = *reinterpret_cast<const bf16x8_t *>(ha + (j + u) * 512);
      b[u] = *reinterpret_cast<const bf16x8_t *>(gb + (j + u) * 512);
    }
#pragma unroll
    for (int u = 0; u < DWP_U; ++u) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u], b[u], acc, 0, 0, 0);
      if (bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cs += (float)b[u][e];
      }
    }
  }
  for (; j < jb; ++j) {
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t *>(ha + j * 512);
    const bf16x8_t b = *reinterpret_cast<const bf16x8_t *>(gb + j * 512);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    if (bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) cs += (float)b[e];
    }
  }
  float *dst = part + ((int64_t)job * S + sp) * DWS_STRIDE;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    reinterpret_cast<float4 *>(dst + lane * 16)[q] = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
  dst[1024 + lane] = cs;
}

__global__ __launch_bounds__(64) void tower_dw_split_reduce_kernel(TowerP p, int S, const float *__restrict__ part) {
  int l, i, k0, n0, row0, nrows;
  const int job = blockIdx.x;
  if (!dw_job(p, job, l, i, k0, n0, row0, nrows)) return;
  int K, N;
  chain_dims(p.d, i, K, N);
  const int lane = threadIdx.x, half = lane >> 5;
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float cs = 0.f;
  for (int sp = 0; sp < S; ++sp) {
    const float *src = part + ((int64_t)job * S + sp) * DWS_STRIDE;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = reinterpret_cast<const float4 *>(src + lane * 16)[q];
      acc[4 * q] += v.x;
      acc[4 * q + 1] += v.y;
      acc[4 * q + 2] += v.z;
      acc[4 * q + 3] += v.w;
    }
    cs += src[1024 + lane];
  }
  float *gw = p.gw[l] + (int64_t)(k0 + 4 * half) * N + n0 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) gw[(int64_t)((r & 3) + 8 * (r >> 2)) * N] = acc[r];
  if (k0 == 0) {
    cs += __shfl_xor(cs, 32);
    if (half == 0) p.gb[l][n0 + lane] = cs;
  }
}

__global__ __launch_bounds__(256) void tower_reduce_kernel(TowerP p) {
  const int nb = p.R / RB, nbB = p.B / RB;
  const int64_t E = p.slab_elems;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
    int i = 0;
    while (i < 5 && e >= slab_off(p.d, i + 1)) ++i;
    int K, N;
    chain_dims(p.d, i, K, N);
    const int64_t o = e - slab_off(p.d, i);
    const bool is_b = o >= (int64_t)K * N;
    if (i < 3) {
      float s = 0.f;
      for (int bk = 0; bk < nb; ++bk) s += p.slab[(int64_t)bk * E + e];
      if (is_b) p.gb[i][o - (int64_t)K * N] = s; else p.gw[i][o] = s;
    } else {
      float s1 = 0.f, s2 = 0.f;
      for (int bk = 0; bk < nbB; ++bk) s1 += p.slab[(int64_t)bk * E + e];
      for (int bk = nbB; bk < nb; ++bk) s2 += p.slab[(int64_t)bk * E + e];
      const int l1 = i, l2 = i + 3;
      if (is_b) {
        p.gb[l1][o - (int64_t)K * N] = s1;
        if (nb > nbB) p.gb[l2][o - (int64_t)K * N] = s2;
      } else {
        p.gw[l1][o] = s1;
        if (nb > nbB) p.gw[l2][o] = s2;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void tower_transpose_kernel(TowerP p, int64_t *state, int64_t bpe) {
  __shared__ T tile[32][33];
  if (state && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {  // cc_state_advance
    state[0] += 1;
    state[1] += 1;
    if (state[1] >= bpe) {
      state[1] = 0;
      state[2] += 1;
    }
  }
  const int l = blockIdx.y;
  const int i = l < 3 ? l : (l < 6 ? l : l - 3);
  int K, N;
  chain_dims(p.d, i, K, N);
  const int tn = N / 32, ntile = (K / 32) * tn;
  const T *w = reinterpret_cast<const T *>(p.w[l]);
  T *wt = reinterpret_cast<T *>(p.wt[l]);
  for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
    const int k0 = 32 * (t / tn), n0 = 32 * (t % tn);
    for (int e = threadIdx.x; e < 1024; e += 256) tile[e / 32][e % 32] = w[(int64_t)(k0 + e / 32) * N + n0 + e % 32];
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 256) wt[(int64_t)(n0 + e / 32) * K + k0 + e % 32] = tile[e % 32][e / 32];
    __syncthreads();
  }
  if constexpr (sizeof(T) == 2) {
    if (p.packed) {  // fragment-packed forward (rows n, reduction k) and backward (rows k, red. n)
      const bf16_t *wb = reinterpret_cast<const bf16_t *>(p.w[l]);
      bf16_t *pf = const_cast<bf16_t *>(p.wpf[l]), *pb = const_cast<bf16_t *>(p.wpb[l]);
      const int nfr = K * N / 8;
      for (int f = blockIdx.x * 256 + threadIdx.x; f < nfr; f += gridDim.x * 256) {
        const int lane = f & 63, q = f >> 6;
        {  // forward: fragment (t, j) over K/16 reduction steps
          const int j = q % (K / 16), tt = q / (K / 16);
          const int n = 32 * tt + (lane & 31), k0 = 16 * j + 8 * (lane >> 5);
          uint16_t e8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) e8[e] = wb[(int64_t)(k0 + e) * N + n];
          *reinterpret_cast<uint4 *>(pf + pack_off(tt, j, lane, K)) = *reinterpret_cast<const uint4 *>(e8);
        }
        {  // backward: fragment (t, j) over N/16 reduction steps, rows are W's rows
          const int j = q % (N / 16), tt = q / (N / 16);
          const int k = 32 * tt + (lane & 31), n0 = 16 * j + 8 * (lane >> 5);
          *reinterpret_cast<uint4 *>(pb + pack_off(tt, j, lane, N)) =
              *reinterpret_cast<const uint4 *>(wb + (int64_t)k * N + n0);
        }
      }
    }
  }
}

int make_params(const cc_tower_args *t, TowerP &p) {
  if (!t) return cc::fail(CC_ERR_ARG, "cc_tower: null args");
  if (t->dtype != CC_BF16 && t->dtype != CC_F32) return cc::fail(CC_ERR_ARG, "cc_tower: dtype");
  const int maxd = t->dtype == CC_BF16 ? 1024 : 256;
  if (t->d < 64 || t->d > maxd || t->d % 64) return cc::fail(CC_ERR_UNSUPPORTED, "cc_tower: d out of range for the fused towers");
  if (t->B % RB || t->R % RB || t->R < t->B || t->B <= 0) return cc::fail(CC_ERR_ARG, "cc_tower: B and R must be multiples of 32");
  p.d = t->d;
  p.B = t->B;
  p.R = t->R;
  p.maxw = t->d > 256 ? t->d : 256;
  for (int l = 0; l < 9; ++l) {
    p.w[l] = t->w[l];
    p.wt[l] = t->wt[l];
    p.b[l] = t->b[l];
    p.gw[l] = t->gw[l];
    p.gb[l] = t->gb[l];
  }
  for (int a = 0; a < 7; ++a) p.act[a] = t->act[a];
  p.act6t = t->act6t;
  p.gD3 = t->gD3;
  for (int a = 0; a < 5; ++a) p.gact[a] = t->gact[a];
  p.gpre1 = t->gpre1;
  p.gpre1t = t->dtype == CC_BF16 ? t->gpre1t : nullptr;
  p.gpre1p = t->dtype == CC_BF16 && t->d <= 256 ? static_cast<bf16_t *>(t->gpre1p) : nullptr;
  p.yb = static_cast<const uint32_t *>(t->y_bits);
  p.yimg = static_cast<uint32_t *>(t->y_img);
  p.y_VW = t->y_V > 0 ? (t->y_V + 31) / 32 : 0;
  p.xb = static_cast<const uint32_t *>(t->x_bits);
  p.xt = static_cast<uint32_t *>(t->xt_bits);
  p.xt_V = t->xt_V;
  p.xt_rows = t->xt_rows;
  // D3's MX-FP8 images: the wide bf16 chains only (all four pointers, 16-B aligned, R % 32 == 0)
  p.d3q = static_cast<uint8_t *>(t->d3q);
  p.d3qs = static_cast<uint8_t *>(t->d3qs);
  p.d3tq = static_cast<uint8_t *>(t->d3tq);
  p.d3tqs = static_cast<uint8_t *>(t->d3tqs);
  if (p.d3q && !(p.d3qs && p.d3tq && p.d3tqs && t->dtype == CC_BF16 && t->d > 256 && t->d % 32 == 0 &&
                 t->R % 32 == 0 && (((uintptr_t)p.d3q | (uintptr_t)p.d3tq) & 15) == 0))
    return cc::fail(CC_ERR_ARG, "cc_tower: d3q/d3qs/d3tq/d3tqs need bf16, 256 < d (d % 32 == 0), R % 32 == 0, 16-B aligned codes");
  if ((uintptr_t)p.gpre1p & 15) return cc::fail(CC_ERR_ARG, "cc_tower: gpre1p must be 16-B aligned");
  p.slab = t->slab;
  p.slab_elems = slab_off(t->d, 6);
  // packed weight images: d <= 256 (fast kernels, optional) and 256 < d <= 1024 (wide kernels,
  // which need them; without them the generic 4-wave kernels run)
  p.packed = t->dtype == CC_BF16;
  for (int l = 0; l < 9; ++l) {
    p.wpf[l] = static_cast<const bf16_t *>(t->wpf[l]);
    p.wpb[l] = static_cast<const bf16_t *>(t->wpb[l]);
    if (l < (t->R > t->B ? 9 : 6) && (!t->wpf[l] || !t->wpb[l])) p.packed = false;
  }
  const bool narrow = t->dtype == CC_BF16 && t->d <= 256;
  const bool fast = narrow || p.packed;  // the fast (d <= 256) or wide chains run
  p.dwpacked = fast;
  for (int a = 0; a < 6; ++a) {
    p.hpt[a] = static_cast<bf16_t *>(t->hpt[a]);
    p.gpt[a] = static_cast<bf16_t *>(t->gpt[a]);
    if (!t->hpt[a] || !t->gpt[a] || (((uintptr_t)t->hpt[a] | (uintptr_t)t->gpt[a]) & 15)) p.dwpacked = false;
  }
  if (t->B % 16 || t->R % 16) p.dwpacked = false;
  // fused D1 / D2 operands: written by the fast (d <= 256) and wide (d <= 1024) bf16 chains
  p.act6p = t->dtype == CC_BF16 && fast ? static_cast<bf16_t *>(t->act6p) : nullptr;
  p.act6tp = t->dtype == CC_BF16 && fast ? static_cast<bf16_t *>(t->act6tp) : nullptr;
  if (((uintptr_t)p.act6p | (uintptr_t)p.act6tp) & 15)
    return cc::fail(CC_ERR_ARG, "cc_tower: packed D3 images must be 16-B aligned");
  if (p.packed)
    for (int l = 0; l < 9; ++l)
      if ((((uintptr_t)t->wpf[l] | (uintptr_t)t->wpb[l]) & 15) != 0)
        return cc::fail(CC_ERR_ARG, "cc_tower: packed weight images must be 16-B aligned");
  return CC_OK;
}

}  // namespace

extern "C" int64_t cc_tower_slab_elems(int32_t d) { return slab_off(d, 6); }

// y_img (the fused D1 kernel's target-mask image) rides in the fast forward only
static int check_yimg(const TowerP &p) {
  CC_REQUIRE(!p.yimg || (p.yb && p.y_VW > 0 && p.d <= 256 && !p.d3q),
             "cc_tower_fwd: y_img needs y_bits, y_V > 0 and the bf16 fast chains (d <= 256)");
  CC_REQUIRE(!p.yimg || (size_t)2 * RB * (p.maxw + 8) * 2 >= (size_t)32 * (YI_W + 1) * 4,
             "cc_tower_fwd: y_img transpose LDS");
  return CC_OK;
}

extern "C" int cc_tower_fwd(const cc_tower_args *t, void *stream) {
  TowerP p;
  int rc = make_params(t, p);
  if (rc) return rc;
  const int es = t->dtype == CC_BF16 ? 2 : 4;
  const size_t lds = (size_t)2 * RB * (p.maxw + 16 / es) * es;
  rc = check_yimg(p);
  if (rc) return rc;
  CC_REQUIRE(!p.yimg || t->dtype == CC_BF16, "cc_tower_fwd: y_img needs the bf16 fast chains");
  CC_REQUIRE(!p.xt || (p.xb && t->dtype == CC_BF16 && p.d <= 256 && p.xt_V > 0 && p.xt_rows >= 1 &&
                       p.xt_rows <= p.R),
             "cc_tower_fwd: xt_bits needs x_bits, bf16, d <= 256 and 1 <= xt_rows <= R");
  if (t->dtype == CC_BF16 && p.d <= 256) {
    const int nxt = p.xt ? (int)cdiv((p.xt_V + 31) / 32, XT_TJ) : 0;
    const int nyi = p.yimg ? yimg_blocks(p.B, p.y_VW) : 0;
    const dim3 g((unsigned)(p.R / RB + nxt + nyi)), b(FNT);
    hipStream_t s = as_stream(stream);
    switch (p.d) {
      case 64: hipLaunchKernelGGL(tower_fwd_fast_kernel<64>, g, b, lds, s, p, nxt); break;
      case 128: hipLaunchKernelGGL(tower_fwd_fast_kernel<128>, g, b, lds, s, p, nxt); break;
      case 192: hipLaunchKernelGGL(tower_fwd_fast_kernel<192>, g, b, lds, s, p, nxt); break;
      default: hipLaunchKernelGGL(tower_fwd_fast_kernel<256>, g, b, lds, s, p, nxt); break;
    }
  }
  else if (t->dtype == CC_BF16 && p.packed)
    hipLaunchKernelGGL(tower_fwd_wide_kernel, dim3(p.R / RB), dim3(FNT), lds, as_stream(stream), p);
  else if (t->dtype == CC_BF16)
    hipLaunchKernelGGL(tower_fwd_kernel<bf16_t>, dim3(p.R / RB), dim3(NT), lds, as_stream(stream), p);
  else
    hipLaunchKernelGGL(tower_fwd_kernel<float>, dim3(p.R / RB), dim3(NT), lds, as_stream(stream), p);
  CC_LAUNCH_CHECK("tower_fwd_kernel");
  return CC_OK;
}

static int tower_bwd_launch(const cc_tower_args *t, void *stream, bool chain, bool dw,
                            const cc_adam::Args *ad = nullptr, const int64_t *ad_state = nullptr,
                            int ad_blocks = 0, const cc_adam::Args *ad1 = nullptr,
                            const cc_noise_args *na = nullptr, int64_t bpe = 1) {
  TowerP p;
  int rc = make_params(t, p);
  if (rc) return rc;
  CC_REQUIRE(t->gD3 && t->gpre1 && t->slab, "cc_tower_bwd: null gD3/gpre1/slab");
  for (int a = 0; a < 5; ++a) CC_REQUIRE(t->gact[a], "cc_tower_bwd: null gact");
  const int es = t->dtype == CC_BF16 ? 2 : 4;
  const size_t lds_chain = (size_t)2 * RB * (p.maxw + 16 / es) * es;
  const size_t lds_dw = (size_t)2 * p.maxw * (RB + 16 / es) * es;
  const dim3 gc(p.R / RB), gd(6 * (p.R / RB));
  hipStream_t s = as_stream(stream);
  if (t->dtype == CC_BF16) {
    if (chain && p.d <= 256) {
      const cc_adam::Args a0 = ad ? *ad : cc_adam::Args{}, a1 = ad1 ? *ad1 : cc_adam::Args{};
      const int nf = na ? (na->B + TF_CPB - 1) / TF_CPB : 0;
      const dim3 ga(gc.x + nf + (ad ? ad_blocks : 0));
      // F's blocks (TF_CPB cubes each): their cube / cut / ycut / add bitmasks and scans in the same
      // dynamic LDS
      const size_t lds_f = na ? (size_t)TF_CPB * (4 * ((na->V + 31) / 32) + FNT / TF_CPB + 1) * 4 : 0;
      const size_t lds_cf = std::max(lds_chain, lds_f);
      const cc_noise_args nn = na ? *na : cc_noise_args{};
#define CHAIN_FAST(DD)                                                                                    \
  if (na && ad)                                                                                           \
    hipLaunchKernelGGL((tower_bwd_chain_fast_kernel<DD, true, true>), ga, dim3(FNT), lds_cf, s, p, a0, a1, \
                       ad_state, nn, bpe);                                                                \
  else if (na)                                                                                            \
    hipLaunchKernelGGL((tower_bwd_chain_fast_kernel<DD, false, true>), ga, dim3(FNT), lds_cf, s, p, a0,    \
                       a1, ad_state, nn, bpe);                                                            \
  else if (ad)                                                                                            \
    hipLaunchKernelGGL((tower_bwd_chain_fast_kernel<DD, true>), ga, dim3(FNT), lds_chain, s, p, a0, a1,    \
                       ad_state, cc_noise_args{}, (int64_t)1);                                            \
  else                                                                                                    \
    hipLaunchKernelGGL((tower_bwd_chain_fast_kernel<DD, false>), gc, dim3(FNT), lds_chain, s, p, a0, a1,   \
                       ad_state, cc_noise_args{}, (int64_t)1);
      switch (p.d) {
        case 64: CHAIN_FAST(64) break;
        case 128: CHAIN_FAST(128) break;
        case 192: CHAIN_FAST(192) break;
        default: CHAIN_FAST(256) break;
      }
#undef CHAIN_FAST
    }
    else if (chain && p.packed)
      hipLaunchKernelGGL(tower_bwd_chain_wide_kernel, gc, dim3(FNT), lds_chain, s, p);
    else if (chain)
      hipLaunchKernelGGL(tower_bwd_chain_kernel<bf16_t>, gc, dim3(NT), lds_chain, s, p);
    if (dw) hipLaunchKernelGGL(tower_dw_kernel<bf16_t>, gd, dim3(NT), lds_dw, s, p);
  } else {
    if (chain) hipLaunchKernelGGL(tower_bwd_chain_kernel<float>, gc, dim3(NT), lds_chain, s, p);
    if (dw) hipLaunchKernelGGL(tower_dw_kernel<float>, gd, dim3(NT), lds_dw, s, p);
  }
  CC_LAUNCH_CHECK("tower_bwd kernels");
  return CC_OK;
}

extern "C" int cc_tower_bwd(const cc_tower_args *t, void *stream) {
  return tower_bwd_launch(t, stream, true, true);
}
extern "C" int cc_tower_bwd_chain(const cc_tower_args *t, void *stream) {
  return tower_bwd_launch(t, stream, true, false);
}
extern "C" int cc_tower_bwd_chain_adam(const cc_tower_args *t, float *p, float *m, float *v, const float *g,
                                       uint16_t *shadow, int64_t lo0, int64_t n0, int64_t lo1, int64_t n1,
                                       const int64_t *state, float lr, float beta1, float beta2, float eps,
                                       void *stream) {
  CC_REQUIRE(t && t->dtype == CC_BF16 && t->d <= 256,
             "cc_tower_bwd_chain_adam: the bf16 fast chains (d <= 256) only");
  CC_REQUIRE(p && m && v && g && state, "cc_tower_bwd_chain_adam: null pointer");
  CC_REQUIRE(((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g) % 16 == 0 && lo0 % 4 == 0 && lo1 % 4 == 0,
             "cc_tower_bwd_chain_adam: buffers must be 16-byte aligned, range starts multiples of 4");
  CC_REQUIRE(!shadow || (uintptr_t)shadow % 8 == 0, "cc_tower_bwd_chain_adam: shadow must be 8-byte aligned");
  CC_REQUIRE(lo0 >= 0 && n0 >= 0 && n1 >= 0 && (n1 == 0 || lo1 >= lo0 + n0), "cc_tower_bwd_chain_adam: ranges");
  const int64_t n = n0 + n1;
  if (n == 0) return tower_bwd_launch(t, stream, true, false);
  const cc_adam::Args a{p + lo0, m + lo0, v + lo0, g + lo0, shadow ? (bf16_t *)shadow + lo0 : nullptr, n0,
                        lr, beta1, beta2, eps, lo0};
  const cc_adam::Args a1{p + lo1, m + lo1, v + lo1, g + lo1, shadow ? (bf16_t *)shadow + lo1 : nullptr, n1,
                         lr, beta1, beta2, eps, lo1};
  // one 512-thread block per CU beside the chains (their VGPR budget admits one per CU), capped
  // so no block runs out of work
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int64_t want = cdiv(cdiv(n, 4), (int64_t)FNT * 4);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(want, std::max(cus - t->R / RB, 8)));
  return tower_bwd_launch(t, stream, true, false, &a, state, blocks, &a1);
}
// the chains + F of the NEXT step (cc_noise_fwd's arguments; {step, batch, epoch} advanced as the
// Adam + F launch does) + optionally TF Adam over [lo0, lo0 + n0) and [lo1, lo1 + n1) (n0 = n1 = 0:
// none), in one launch
extern "C" int cc_tower_bwd_chain_noise(const cc_tower_args *t, const cc_noise_args *next, int64_t batches_per_epoch,
                                        float *p, float *m, float *v, const float *g, uint16_t *shadow,
                                        int64_t lo0, int64_t n0, int64_t lo1, int64_t n1, const int64_t *state,
                                        float lr, float beta1, float beta2, float eps, void *stream) {
  CC_REQUIRE(t && t->dtype == CC_BF16 && t->d <= 256,
             "cc_tower_bwd_chain_noise: the bf16 fast chains (d <= 256) only");
  CC_REQUIRE(next && next->V > 0 && next->B > 0 && next->x_cap > 0 && next->cube_ptr && next->cube_idx &&
                 next->perm && next->cdf && next->neg_sampler && next->state && next->x_cnt && next->x_idx &&
                 next->y_bits && next->status && (!next->with_reg || next->reg_idx),
             "cc_tower_bwd_chain_noise: F arguments");
  CC_REQUIRE(next->xt_bits == nullptr,
             "cc_tower_bwd_chain_noise: F may not set xt bits here (the W1 gradient still reads them)");
  CC_REQUIRE(next->num_perms >= 1 && next->num_cubes >= next->batch_stride && batches_per_epoch >= 1,
             "cc_tower_bwd_chain_noise: num_perms / num_cubes / batches_per_epoch");
  CC_REQUIRE((size_t)TF_CPB * (4 * ((next->V + 31) / 32) + FNT / TF_CPB + 1) * 4 <= 150 * 1024,
             "cc_tower_bwd_chain_noise: V too large");
  const int64_t n = n0 + n1;
  if (n == 0)
    return tower_bwd_launch(t, stream, true, false, nullptr, nullptr, 0, nullptr, next, batches_per_epoch);
  CC_REQUIRE(p && m && v && g && state, "cc_tower_bwd_chain_noise: null Adam pointer");
  CC_REQUIRE(((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g) % 16 == 0 && lo0 % 4 == 0 && lo1 % 4 == 0,
             "cc_tower_bwd_chain_noise: buffers must be 16-byte aligned, range starts multiples of 4");
  CC_REQUIRE(!shadow || (uintptr_t)shadow % 8 == 0, "cc_tower_bwd_chain_noise: shadow must be 8-byte aligned");
  CC_REQUIRE(lo0 >= 0 && n0 >= 0 && n1 >= 0 && (n1 == 0 || lo1 >= lo0 + n0), "cc_tower_bwd_chain_noise: ranges");
  const cc_adam::Args a{p + lo0, m + lo0, v + lo0, g + lo0, shadow ? (bf16_t *)shadow + lo0 : nullptr, n0,
                        lr, beta1, beta2, eps, lo0};
  const cc_adam::Args a1{p + lo1, m + lo1, v + lo1, g + lo1, shadow ? (bf16_t *)shadow + lo1 : nullptr, n1,
                         lr, beta1, beta2, eps, lo1};
  const int64_t want = cdiv(cdiv(n, 4), (int64_t)FNT * 4);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(want, 256));
  return tower_bwd_launch(t, stream, true, false, &a, state, blocks, &a1, next, batches_per_epoch);
}

extern "C" int cc_tower_bwd_dw(const cc_tower_args *t, void *stream) {
  return tower_bwd_launch(t, stream, false, true);
}

extern "C" int cc_tower_reduce(const cc_tower_args *t, void *stream) {
  TowerP p;
  int rc = make_params(t, p);
  if (rc) return rc;
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv(p.slab_elems, 256), 2048);
  hipLaunchKernelGGL(tower_reduce_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), p);
  CC_LAUNCH_CHECK("tower_reduce_kernel");
  return CC_OK;
}

extern "C" int cc_tower_bwd_dw_direct(const cc_tower_args *t, void *stream) {
  TowerP p;
  int rc = make_params(t, p);
  if (rc) return rc;
  CC_REQUIRE(t->dtype == CC_BF16, "cc_tower_bwd_dw_direct: bf16 only");
  CC_REQUIRE(t->gD3, "cc_tower_bwd_dw_direct: null gD3");
  for (int a = 0; a < 5; ++a) CC_REQUIRE(t->gact[a], "cc_tower_bwd_dw_direct: null gact");
  for (int l = 0; l < (t->R > t->B ? 9 : 6); ++l)
    CC_REQUIRE(t->gw[l] && t->gb[l], "cc_tower_bwd_dw_direct: null gw/gb");
  const int rmax = t->R > t->B ? t->R : t->B;
  const int rpw = ((rmax + 3) / 4 + 15) / 16 * 16;
  const size_t lds = std::max((size_t)4 * 2 * 32 * (rpw + 8) * 2, (size_t)(4 * 32 * 33 + 4 * 32) * 4);
  int jobs = 0;
  for (int l = 0; l < (t->R > t->B ? 9 : 6); ++l) {
    int K, N;
    chain_dims(t->d, l < 6 ? l : l - 3, K, N);
    jobs += (K / 32) * (N / 32);
  }
  if (p.dwpacked) {  // the forward / backward chains wrote the packed transposed H_i / G_i
    // tall chains (full-mode regulariser rows): split the rows, S partials per tile in the slab
    const int S = std::min(16, std::max(1, t->R / 1024));
    if (S > 1 && p.slab && (int64_t)jobs * S * DWS_STRIDE <= (int64_t)(t->R / RB) * p.slab_elems) {
      hipLaunchKernelGGL(tower_dw_packed_split_kernel, dim3(jobs, S), dim3(64), 0, as_stream(stream), p, S, p.slab);
      CC_LAUNCH_CHECK("tower_dw_packed_split_kernel");
      hipLaunchKernelGGL(tower_dw_split_reduce_kernel, dim3(jobs), dim3(64), 0, as_stream(stream), p, S, p.slab);
      CC_LAUNCH_CHECK("tower_dw_split_reduce_kernel");
      return CC_OK;
    }
    hipLaunchKernelGGL(tower_dw_packed_kernel, dim3(jobs), dim3(64), 0, as_stream(stream), p);
    CC_LAUNCH_CHECK("tower_dw_packed_kernel");
    return CC_OK;
  }
  CC_REQUIRE(lds <= 160 * 1024, "cc_tower_bwd_dw_direct: too many rows for one LDS stage (use cc_tower_bwd_dw)");
  hipLaunchKernelGGL(tower_dw_tiled_kernel, dim3(jobs), dim3(DW_NT), lds, as_stream(stream), p, rpw);
  CC_LAUNCH_CHECK("tower_dw_tiled_kernel");
  return CC_OK;
}

extern "C" int cc_tower_transpose_advance(const cc_tower_args *t, int64_t *state,
                                          int64_t batches_per_epoch, void *stream) {
  TowerP p;
  int rc = make_params(t, p);
  if (rc) return rc;
  CC_REQUIRE(!state || batches_per_epoch >= 1, "cc_tower_transpose_advance: batches_per_epoch");
  const int layers = t->R > t->B ? 9 : 6;
  if (t->dtype == CC_BF16)
    hipLaunchKernelGGL(tower_transpose_kernel<bf16_t>, dim3(64, layers), dim3(256), 0, as_stream(stream), p,
                       state, batches_per_epoch);
  else
    hipLaunchKernelGGL(tower_transpose_kernel<float>, dim3(64, layers), dim3(256), 0, as_stream(stream), p,
                       state, batches_per_epoch);
  CC_LAUNCH_CHECK("tower_transpose_kernel");
  return CC_OK;
}

extern "C" int cc_tower_transpose(const cc_tower_args *t, void *stream) {
  return cc_tower_transpose_advance(t, nullptr, 1, stream);
}
