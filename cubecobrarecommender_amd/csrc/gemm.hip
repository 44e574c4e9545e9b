// Generic LDS-staged MFMA GEMM with fused epilogues — the Dense layers of the encoder and
// decoder towers (model.py:29-33, 58-62), the decoder output layers (model.py:64) and their
// backward products.  C[M,N] = op(A)[M,K] op(B)[K,N], fp32 accumulation.
//
//   bf16 operands: v_mfma_f32_32x32x16_bf16   (lane l: A[l&31][8(l>>5)+j], B[8(l>>5)+j][l&31])
//   fp32 operands: v_mfma_f32_32x32x2_f32     (lane l: A[l&31][l>>5],       B[l>>5][l&31]) —
//                  exact fp32 (a k-ordered fmaf chain), used for the fp32 parity mode.
// Workgroup = 4 waves (256 threads), 64x64 output tile, 2x2 waves of 32x32, BK = 32/64/128 by K.
// Both LDS images are K-contiguous ([row][k] / [col][k]); transposed global layouts are
// transposed during staging so every fragment read is one ds_read_b128 (bf16) / b32 (fp32).
// Accumulator map (32x32): row = (r&3) + 8(r>>2) + 4(l>>5), col = l&31.
#include <cstdlib>

#include "common.hpp"

// build knobs (A/B builds: CCREC_EXTRA_FLAGS=-D..., a tagged library; the library reads no environment)
#ifndef CCREC_NT_BM
#define CCREC_NT_BM 0
#endif
#ifndef CCREC_GEMM_NT
#define CCREC_GEMM_NT 1
#endif

namespace {

constexpr int BM = 64, BN = 64, NT = 256;

struct GemmParams {
  int M, N, K, lda, ldb, ldc, splits, relu;
  int vec_a, vec_b;
  const void *A, *B;
  const float *bias;
  void *C;
  float *Cf;
  const void *H;
  const uint32_t *y_bits;
  float scale;
  double *loss_partials;
  float *colsum;
  void *Ct;
  int ldct;
  double *loss_out;
  double loss_scale;
  uint32_t *ticket;
  const uint8_t *sa, *sb;  // MX-FP8: E8M0 block scales [M][lda/32], [N][ldb/32]
};

template <typename T> struct Mma;
template <> struct Mma<bf16_t> {
  static constexpr int KM = 16;
  static __device__ __forceinline__ void step(const bf16_t *a_row, const bf16_t *b_row, int kk,
                                              int half, f32x16_t &acc) {
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t *>(a_row + kk + 8 * half);
    const bf16x8_t b = *reinterpret_cast<const bf16x8_t *>(b_row + kk + 8 * half);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int KM = 2;
  static __device__ __forceinline__ void step(const float *a_row, const float *b_row, int kk,
                                              int half, f32x16_t &acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a_row[kk + half], b_row[kk + half], acc, 0, 0, 0);
  }
};

// Register-staged tile loader for a ROWS x BK tile of the logical operand X[row][k]
// (row in [r0, r0+ROWS), k in [k0, kend)) into the K-contiguous LDS image S[row][k].
//   KCONTIG: storage X[row*ld + k] (16-B vectors along k, stored to LDS as one b128);
//   else   : storage X[k*ld + row] (16-B vectors along row, transposed into LDS element-wise).
// load() issues the global loads into registers; store() writes them to LDS — split so the next
// tile's loads are in flight while the current tile's MFMAs run.
template <typename T, bool KCONTIG, int ROWS, int BK>
struct Stager {
  static constexpr int VW = 16 / sizeof(T);
  static constexpr int NVEC = ROWS * BK / VW;
  static constexpr int NV = (NVEC + NT - 1) / NT;
  uint4 r[NV];

  __device__ __forceinline__ void load(const T *__restrict__ X, int ld, int r0, int rlim, int k0,
                                       int kend, bool vec_ok) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = threadIdx.x + i * NT;
      if (v >= NVEC) break;
      int gr, gk;
      bool full;
      const T *src;
      if constexpr (KCONTIG) {
        constexpr int PER = BK / VW;
        gr = r0 + v / PER;
        gk = k0 + (v % PER) * VW;
        full = vec_ok && gr < rlim && gk + VW <= kend;
        src = X + (int64_t)gr * ld + gk;
      } else {
        constexpr int PER = ROWS / VW;
        gk = k0 + v / PER;
        gr = r0 + (v % PER) * VW;
        full = vec_ok && gk < kend && gr + VW <= rlim;
        src = X + (int64_t)gk * ld + gr;
      }
      if (full) {
        r[i] = *reinterpret_cast<const uint4 *>(src);
      } else {
        T tmp[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          const bool ok = KCONTIG ? (gr < rlim && gk + e < kend) : (gk < kend && gr + e < rlim);
          tmp[e] = ok ? src[e * (KCONTIG ? 1 : 1)] : T(0);
        }
        r[i] = *reinterpret_cast<const uint4 *>(tmp);
      }
    }
  }

  template <int LDK>
  __device__ __forceinline__ void store(T (*S)[LDK]) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = threadIdx.x + i * NT;
      if (v >= NVEC) break;
      if constexpr (KCONTIG) {
        constexpr int PER = BK / VW;
        *reinterpret_cast<uint4 *>(&S[v / PER][(v % PER) * VW]) = r[i];
      } else {
        constexpr int PER = ROWS / VW;
        const int k = v / PER, rv = (v % PER) * VW;
        const T *tmp = reinterpret_cast<const T *>(&r[i]);
#pragma unroll
        for (int e = 0; e < VW; ++e) S[rv + e][k] = tmp[e];
      }
    }
  }
};

__device__ __forceinline__ double block_sum_double(double v, double *red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < NT / 64; ++w) s += red[w];
  return s;
}

template <typename T, bool TA, bool TB, int EPI, int BK>
__global__ __launch_bounds__(NT) void gemm_kernel(GemmParams p) {
  constexpr int PADK = 16 / sizeof(T);
  constexpr int LDK = BK + PADK;
  __shared__ __attribute__((aligned(16))) T As[BM][LDK];
  __shared__ __attribute__((aligned(16))) T Bs[BN][LDK];
  __shared__ double red[NT / 64];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bm = blockIdx.y * BM, bn = blockIdx.x * BN;
  int kbeg = 0, kend = p.K;
  if constexpr (EPI == CC_EPI_SPLITK) {
    const int kchunk = (int)cdiv(cdiv(p.K, p.splits), BK) * BK;
    kbeg = blockIdx.z * kchunk;
    kend = min(p.K, kbeg + kchunk);
  }
  const T *__restrict__ A = reinterpret_cast<const T *>(p.A);
  const T *__restrict__ B = reinterpret_cast<const T *>(p.B);
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const T *a_row = &As[wm * 32 + (lane & 31)][0];
  const T *b_row = &Bs[wn * 32 + (lane & 31)][0];
  const int half = lane >> 5;
  // fused bias gradient: the first row of blocks sums the staged op(B) tile over k (ascending)
  const bool do_cs = p.colsum != nullptr && blockIdx.y == 0 && threadIdx.x < BN;
  float cs = 0.f;
  Stager<T, !TA, BM, BK> sa;
  Stager<T, TB, BN, BK> sb;
  if (kbeg < kend) {
    sa.load(A, p.lda, bm, p.M, kbeg, kend, p.vec_a);
    sb.load(B, p.ldb, bn, p.N, kbeg, kend, p.vec_b);
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    sa.store(As);
    sb.store(Bs);
    __syncthreads();
    if (k0 + BK < kend) {  // next tile's global loads fly while this tile's MFMAs run
      sa.load(A, p.lda, bm, p.M, k0 + BK, kend, p.vec_a);
      sb.load(B, p.ldb, bn, p.N, k0 + BK, kend, p.vec_b);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += Mma<T>::KM) Mma<T>::step(a_row, b_row, kk, half, acc);
    if (do_cs) {
#pragma unroll 8
      for (int k = 0; k < BK; ++k) cs += DT<T>::ld(&Bs[threadIdx.x][k]);
    }
    __syncthreads();
  }
  if (do_cs && bn + (int)threadIdx.x < p.N) {
    // split-K: one partial row per split (reduced in cc_splitk_reduce)
    const int64_t zo = EPI == CC_EPI_SPLITK ? (int64_t)blockIdx.z * p.N : 0;
    p.colsum[zo + bn + threadIdx.x] = cs;
  }

  // ------------------------------------------------------------------ epilogues
  const int gn = bn + wn * 32 + (lane & 31);
  float lossf = 0.f;
  float dzv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int gm = bm + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
    if (gm >= p.M || gn >= p.N) continue;
    const float a = acc[r];
    if constexpr (EPI == CC_EPI_SPLITK) {
      p.Cf[((int64_t)blockIdx.z * p.M + gm) * p.N + gn] = a;
    } else if constexpr (EPI == CC_EPI_STORE) {
      float v = a + (p.bias ? p.bias[gn] : 0.f);
      if (p.relu) v = v > 0.f ? v : 0.f;
      const int64_t o = (int64_t)gm * p.ldc + gn;
      if (p.C) DT<T>::st(reinterpret_cast<T *>(p.C) + o, v);
      if (p.Cf) p.Cf[o] = v;
    } else if constexpr (EPI == CC_EPI_MASK) {
      const int64_t o = (int64_t)gm * p.ldc + gn;
      const float h = DT<T>::ld(reinterpret_cast<const T *>(p.H) + o);
      const float v = h > 0.f ? a : 0.f;
      if (p.C) DT<T>::st(reinterpret_cast<T *>(p.C) + o, v);
      if (p.Cf) p.Cf[o] = v;
    } else if constexpr (EPI == CC_EPI_BCE) {
      // sigmoid_cross_entropy_with_logits (TF 2.5 Keras BCE on a Sigmoid output)
      const float z = a + p.bias[gn];
      const int YW = (p.N + 31) >> 5;
      const float y = (float)((p.y_bits[(int64_t)gm * YW + (gn >> 5)] >> (gn & 31)) & 1u);
      const float e = __expf(-fabsf(z));               // in (0, 1]
      const float rp = __fdividef(1.f, 1.f + e);
      lossf += fmaxf(z, 0.f) - z * y + __logf(1.f + e);   // log1p(exp(-|z|))
      const float sig = z >= 0.f ? rp : e * rp;
      const float dz = (sig - y) * p.scale;
      dzv[r] = dz;
      const int64_t o = (int64_t)gm * p.ldc + gn;
      if (p.C) DT<T>::st(reinterpret_cast<T *>(p.C) + o, dz);
      if (p.Cf) p.Cf[o] = dz;
    }
  }
  if constexpr (EPI == CC_EPI_BCE) {
    // transposed copy dZ^T [N][M] (k-contiguous operand of the dW = H^T dZ product): registers
    // 4g..4g+3 hold 4 consecutive rows of one column -> one 8-byte (bf16) / 16-byte (fp32) store
    if (p.Ct && gn < p.N) {
      T *ct = reinterpret_cast<T *>(p.Ct) + (int64_t)gn * p.ldct;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row0 = bm + wm * 32 + 8 * g + 4 * half;
        if (row0 + 3 < p.M && (p.ldct & 3) == 0) {
          T v4[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) DT<T>::st(&v4[e], dzv[4 * g + e]);
          if constexpr (sizeof(T) == 2)
            *reinterpret_cast<uint2 *>(ct + row0) = *reinterpret_cast<const uint2 *>(v4);
          else
            *reinterpret_cast<uint4 *>(ct + row0) = *reinterpret_cast<const uint4 *>(v4);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (row0 + e < p.M) DT<T>::st(ct + row0 + e, dzv[4 * g + e]);
        }
      }
    }
    const double s = block_sum_double((double)lossf, red);
    if (threadIdx.x == 0) p.loss_partials[blockIdx.y * gridDim.x + blockIdx.x] = s;
  }
}

// ------------------------------------------------------------------ NT bf16 kernel
// C = A B^T with both operands K-contiguous (A [M][K], B [N][K]) — the decoder output layer's
// forward (D3 Wo^T), weight gradient (D3^T dZ via D3^T and dZ^T images) and input gradient
// (dZ Wo^T, split-K).  BM x 128 tiles (BM = 128/256/512), BM/32 waves each owning 64x64 (2x2
// blocks of v_mfma_f32_32x32x16_bf16); with the decoder's M <= 512 one workgroup covers every row
// of a 128-column panel, so each panel of Wo / dZ^T is read once and the per-tile fixed cost
// (prologue, epilogue) is paid BM/128 times less often.  LDS double-buffered (one barrier per
// K-step; the next K-tile's global loads are in flight during the current tile's MFMAs).  LDS
// rows hold BK bf16 = CH x 16 B chunks stored at chunk ^ (row & (CH-1)), so the rows a fragment
// read touches spread over the banks.  Tiles are assigned XCD-aware: each XCD gets a contiguous
// run, walking M fastest, so the M-tiles sharing one B panel hit the same L2.
// Epilogue: post-op fp32 tile -> LDS (in passes of <= 256 rows) -> 16-B coalesced stores of
// C / Cf rows and of C^T rows (BCE: dZ^T, the k-contiguous operand of dW = D3^T dZ).
constexpr int NBN = 128;
constexpr int SLD = NBN + 1;  // odd row pitch: column reads for C^T spread over the banks
#ifndef NT_RING
#define NT_RING 2
#endif

// T = bf16_t (v_mfma_f32_32x32x16_bf16) or uint8_t = MX-FP8 e4m3 codes with one E8M0 scale per
// 32 K-elements of a row (v_mfma_scale_f32_32x32x64_f8f6f4).  A K-tile is 128 bytes of every row
// either way (64 bf16 / 128 fp8), so staging, swizzle and LDS footprint are shared.
template <int BM, typename T = bf16_t>
struct NtCfg {
  static constexpr bool MX = sizeof(T) == 1;
  static constexpr int NTH = BM * 2;         // BM/32 waves of 64x64 outputs
  static constexpr int BKB = BM >= 512 ? 64 : 128;   // bytes per row per K-tile
  static constexpr int EPC = 16 / (int)sizeof(T);    // elements per 16-B chunk
  static constexpr int BK = BKB / (int)sizeof(T);    // elements per K-tile
  static constexpr int CH = BKB / 16;         // 16-B chunks per LDS row
  static constexpr int A_CH = BM * CH, B_CH = NBN * CH;
  static constexpr int NA = (A_CH + NTH - 1) / NTH, NB = (B_CH + NTH - 1) / NTH;
  static constexpr int STAGE = (BM + NBN) * BKB;    // bytes per K-tile (A + B)
  static constexpr int SCL = MX ? 2 * (BM + NBN) * 4 : 0;  // scale words, double-buffered
  static constexpr int SR = BM > 256 ? 256 : BM;     // rows per epilogue staging pass
  static constexpr int LDS = 2 * STAGE + SCL > SR * SLD * 4 ? 2 * STAGE + SCL : SR * SLD * 4;
};

__device__ __forceinline__ int xcd_tile(int b, int nb) {
  const int q = nb / 8, r = nb % 8, x = b % 8, slot = b / 8;
  return x < r ? x * (q + 1) + slot : r * (q + 1) + (x - r) * q + slot;
}

// Per-thread staging plan, computed once: which 16-B chunks of the A/B tiles this thread moves,
// their global element offsets at k = 0 (rows clamped at the edge: those rows only feed
// discarded outputs) and their swizzled LDS offsets.  The K loop then only adds k0.  MX: thread
// t < BM (< 128) also moves row t's scale word of A (B) — the 4 E8M0 bytes of the K-tile.
template <int BM, typename T = bf16_t>
struct NtPlan {
  using C = NtCfg<BM, T>;
  int64_t ga[C::NA], gb[C::NB];
  int la[C::NA], lb[C::NB];
  int64_t gsa, gsb;
  __device__ __forceinline__ NtPlan(const GemmParams &p, int bm, int bn) {
#pragma unroll
    for (int i = 0; i < C::NA; ++i) {
      const int v = min((int)threadIdx.x + C::NTH * i, C::A_CH - 1), row = v / C::CH, ch = v % C::CH;
      ga[i] = (int64_t)min(bm + row, p.M - 1) * p.lda + ch * C::EPC;
      la[i] = row * C::BK + ((ch ^ (row & (C::CH - 1))) * C::EPC);
    }
#pragma unroll
    for (int i = 0; i < C::NB; ++i) {
      const int v = min((int)threadIdx.x + C::NTH * i, C::B_CH - 1), row = v / C::CH, ch = v % C::CH;
      gb[i] = (int64_t)min(bn + row, p.N - 1) * p.ldb + ch * C::EPC;
      lb[i] = row * C::BK + ((ch ^ (row & (C::CH - 1))) * C::EPC);
    }
    if constexpr (C::MX) {
      const int t = (int)threadIdx.x;
      gsa = (int64_t)min(bm + min(t, BM - 1), p.M - 1) * (p.lda / 32);
      gsb = (int64_t)min(bn + min(t, NBN - 1), p.N - 1) * (p.ldb / 32);
    }
  }
};

template <int BM, typename T = bf16_t>
struct NtStage {
  using C = NtCfg<BM, T>;
  uint4 a[C::NA], b[C::NB];
  uint32_t sa, sb;
  static __device__ __forceinline__ uint4 edge(const T *src, int k, int kend) {
    T tmp[C::EPC];
#pragma unroll
    for (int e = 0; e < C::EPC; ++e) tmp[e] = k + e < kend ? src[e] : (T)0;
    return *reinterpret_cast<const uint4 *>(tmp);
  }
  __device__ __forceinline__ void load(const NtPlan<BM, T> &pl, const T *A, const T *B,
                                       const GemmParams &p, int k0, int kend) {
    if constexpr (C::MX) {  // K % 128 == 0 on this path: whole K-tiles, whole scale words
      if ((int)threadIdx.x < BM) sa = *reinterpret_cast<const uint32_t *>(p.sa + pl.gsa + k0 / 32);
      if ((int)threadIdx.x < NBN) sb = *reinterpret_cast<const uint32_t *>(p.sb + pl.gsb + k0 / 32);
    }
    if (k0 + C::BK <= kend) {  // whole K-tile inside [.., kend): plain 16-B loads
#pragma unroll
      for (int i = 0; i < C::NA; ++i) a[i] = *reinterpret_cast<const uint4 *>(A + pl.ga[i] + k0);
#pragma unroll
      for (int i = 0; i < C::NB; ++i) b[i] = *reinterpret_cast<const uint4 *>(B + pl.gb[i] + k0);
      return;
    }
#pragma unroll
    for (int i = 0; i < C::NA; ++i) {
      const int kc = k0 + (int)((threadIdx.x + C::NTH * i) % C::CH) * C::EPC;
      a[i] = kc + C::EPC <= kend ? *reinterpret_cast<const uint4 *>(A + pl.ga[i] + k0)
                                 : edge(A + pl.ga[i] + k0, kc, kend);
    }
#pragma unroll
    for (int i = 0; i < C::NB; ++i) {
      const int kc = k0 + (int)((threadIdx.x + C::NTH * i) % C::CH) * C::EPC;
      b[i] = kc + C::EPC <= kend ? *reinterpret_cast<const uint4 *>(B + pl.gb[i] + k0)
                                 : edge(B + pl.gb[i] + k0, kc, kend);
    }
  }
  __device__ __forceinline__ void store(const NtPlan<BM, T> &pl, T *As, T *Bs, uint32_t *Ss) const {
#pragma unroll
    for (int i = 0; i < C::NA; ++i)
      if (C::A_CH % C::NTH == 0 || (int)threadIdx.x + C::NTH * i < C::A_CH)
        *reinterpret_cast<uint4 *>(As + pl.la[i]) = a[i];
#pragma unroll
    for (int i = 0; i < C::NB; ++i)
      if (C::B_CH % C::NTH == 0 || (int)threadIdx.x + C::NTH * i < C::B_CH)
        *reinterpret_cast<uint4 *>(Bs + pl.lb[i]) = b[i];
    if constexpr (C::MX) {
      if ((int)threadIdx.x < BM) Ss[threadIdx.x] = sa;
      if ((int)threadIdx.x < NBN) Ss[BM + threadIdx.x] = sb;
    }
  }
};

// MX-FP8 fragment of the 32x32x64 block-scaled MFMA.  The instruction's K order (probed on
// gfx950, a one-off probe of round 3): lane half h holds k 16h .. 16h+15 in its low 16 bytes and
// 32+16h .. 32+16h+15 in its high 16 bytes, and lane half h's scale byte covers k 32h .. 32h+31.
// So for scale block b = 2kk + h of the K-tile, lane half g loads 16-B chunks 4kk + g (low) and
// 4kk + 2 + g (high): chunks {4kk, 4kk+1} form block 2kk, {4kk+2, 4kk+3} block 2kk + 1.
typedef __attribute__((ext_vector_type(4))) int nt_i32x4_t;
typedef __attribute__((ext_vector_type(8))) int nt_i32x8_t;
__device__ __forceinline__ nt_i32x8_t nt_frag8(const uint8_t *S, int row, int c0) {
  constexpr int BKB = 128, CH = 8;
  const nt_i32x4_t lo = *reinterpret_cast<const nt_i32x4_t *>(S + row * BKB + ((c0 ^ (row & (CH - 1))) * 16));
  const nt_i32x4_t hi =
      *reinterpret_cast<const nt_i32x4_t *>(S + row * BKB + (((c0 + 2) ^ (row & (CH - 1))) * 16));
  return nt_i32x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int BK>
__device__ __forceinline__ bf16x8_t nt_frag(const bf16_t *S, int row, int c) {
  return *reinterpret_cast<const bf16x8_t *>(S + row * BK + ((c ^ (row & (BK / 8 - 1))) * 8));
}

// sigmoid_cross_entropy_with_logits (TF 2.5 Keras BCE on a Sigmoid output): returns
// dz = (sigmoid(z) - y) * scale and adds the element's loss when `live`.
__device__ __forceinline__ float bce_dz(float z, uint32_t ybit, float scale, float &loss, bool live) {
  const float y = (float)ybit;
  const float e = __expf(-fabsf(z));  // in (0, 1]
  const float rp = __fdividef(1.f, 1.f + e);
  if (live) loss += fmaxf(z, 0.f) - z * y + __logf(1.f + e);  // log1p(exp(-|z|))
  const float sig = z >= 0.f ? rp : e * rp;
  return (sig - y) * scale;
}

// One output tile of one problem: block `bid` of the problem's `nblk` tile blocks, K split
// `split`; the LDS arrays come from the launching kernel (so two problems sharing a launch do
// not double the LDS).
template <int EPI, int BM, typename T = bf16_t>
__device__ __forceinline__ void nt_body(const GemmParams &p, int tiles_m, int bid, int nblk,
                                        int split, char *smem, uint32_t (*ys)[NBN / 32],
                                        double *red, int &lastflag, bool mapped = false) {
  using C = NtCfg<BM, T>;
  constexpr bool kBceRegs = BM <= 128;  // BCE math on the accumulators (no register pressure)
  constexpr int BK = C::BK, NTH = C::NTH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int tile = mapped ? bid : xcd_tile(bid, nblk);
  // BCE: block-sum the loss and publish it as this tile's partial; with loss_out, an sc1 store
  // + agent ticket (MI355X guide hand-off: no L2 writeback fence) tells the last block to reduce.
  // Called before the epilogue's global stores, so the vmcnt wait has nothing else to drain.
  auto bce_publish = [&](float lf) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) lf += __shfl_xor(lf, off);
    if (lane == 0) red[wave] = (double)lf;
    __syncthreads();
    if (threadIdx.x == 0) {
      double sum = 0.0;
      for (int w = 0; w < NTH / 64; ++w) sum += red[w];
      lastflag = 0;
      if (!p.loss_out) {
        p.loss_partials[tile] = sum;
      } else {
        __hip_atomic_store(&p.loss_partials[tile], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t tk = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lastflag = tk == (uint32_t)nblk - 1;
      }
    }
  };
  const int bm = (tile % tiles_m) * BM, bn = (tile / tiles_m) * NBN;
  int kbeg = 0, kend = p.K;
  if constexpr (EPI == CC_EPI_SPLITK) {
    const int kchunk = (int)cdiv(cdiv(p.K, p.splits), BK) * BK;
    kbeg = split * kchunk;
    kend = min(p.K, kbeg + kchunk);
  }
  if constexpr (EPI == CC_EPI_BCE) {  // lands during the K loop
    const int YW = (p.N + 31) >> 5;
    for (int i = threadIdx.x; i < BM * (NBN / 32); i += NTH) {
      const int r = i / (NBN / 32), w = i % (NBN / 32);
      const int gm = bm + r, gw = (bn >> 5) + w;
      ys[r][w] = gm < p.M && gw < YW ? p.y_bits[(int64_t)gm * YW + gw] : 0u;
    }
  }
  T *AsBase = reinterpret_cast<T *>(smem);
  T *BsBase = AsBase + 2 * BM * BK;
  uint32_t *SsBase = reinterpret_cast<uint32_t *>(smem + 2 * C::STAGE);  // MX: [2][BM + NBN]
  const T *__restrict__ A = reinterpret_cast<const T *>(p.A);
  const T *__restrict__ B = reinterpret_cast<const T *>(p.B);
  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const bool do_cs = !C::MX && p.colsum != nullptr && bm == 0 && threadIdx.x < NBN;
  float cs = 0.f;
  // D-deep register ring: K-tiles t+1 .. t+D-1 are in flight while tile t's MFMAs run; LDS is
  // double-buffered: tile t lives in buffer t & 1.
  constexpr int D = NT_RING;
  const NtPlan<BM, T> pl(p, bm, bn);
  NtStage<BM, T> st[D];
  const int nk = kbeg < kend ? (int)cdiv(kend - kbeg, BK) : 0;
#pragma unroll
  for (int q = 0; q < D; ++q)
    if (q < nk) st[q].load(pl, A, B, p, kbeg + q * BK, kend);
  if (nk > 0) st[0].store(pl, AsBase, BsBase, SsBase);
  __syncthreads();
  const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31);
  for (int t0 = 0; t0 < nk; t0 += D) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const int t = t0 + q;
      if (t >= nk) break;
      const T *as = AsBase + (t & 1) * BM * BK, *bs = BsBase + (t & 1) * NBN * BK;
      if constexpr (C::MX) {
        const uint32_t *ss = SsBase + (t & 1) * (BM + NBN);
        const uint32_t wa0 = ss[ar], wa1 = ss[ar + 32], wb0 = ss[BM + br], wb1 = ss[BM + br + 32];
#pragma unroll
        for (int kk = 0; kk < BK / 64; ++kk) {
          const int c0 = 4 * kk + half, sh = 8 * (2 * kk + half);
          const uint8_t *as8 = reinterpret_cast<const uint8_t *>(as);
          const uint8_t *bs8 = reinterpret_cast<const uint8_t *>(bs);
          const nt_i32x8_t a0 = nt_frag8(as8, ar, c0), a1 = nt_frag8(as8, ar + 32, c0);
          const nt_i32x8_t b0 = nt_frag8(bs8, br, c0), b1 = nt_frag8(bs8, br + 32, c0);
          const int sa0 = (int)((wa0 >> sh) & 0xFFu), sa1 = (int)((wa1 >> sh) & 0xFFu);
          const int sb0 = (int)((wb0 >> sh) & 0xFFu), sb1 = (int)((wb1 >> sh) & 0xFFu);
          acc[0][0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, b0, acc[0][0], 0, 0, 0, sa0, 0, sb0);
          acc[0][1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, b1, acc[0][1], 0, 0, 0, sa0, 0, sb1);
          acc[1][0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, b0, acc[1][0], 0, 0, 0, sa1, 0, sb0);
          acc[1][1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, b1, acc[1][1], 0, 0, 0, sa1, 0, sb1);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
          const int c = 2 * kk + half;
          const bf16x8_t a0 = nt_frag<BK>(as, ar, c), a1 = nt_frag<BK>(as, ar + 32, c);
          const bf16x8_t b0 = nt_frag<BK>(bs, br, c), b1 = nt_frag<BK>(bs, br + 32, c);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (do_cs) {  // bias gradient: sum of B row n over k, ascending k
          const int n = threadIdx.x;
#pragma unroll
          for (int c = 0; c < BK / 8; ++c) {
            const bf16_t *qq = reinterpret_cast<const bf16_t *>(bs) + n * BK + ((c ^ (n & (BK / 8 - 1))) * 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) cs += bf2f(qq[e]);
          }
        }
      }
      // slot q held tile t (already in LDS); refill it with tile t + D, publish tile t + 1
      if (t + D < nk) st[q].load(pl, A, B, p, kbeg + (t + D) * BK, kend);
      if (t + 1 < nk)
        st[(q + 1) % D].store(pl, AsBase + ((t + 1) & 1) * BM * BK, BsBase + ((t + 1) & 1) * NBN * BK,
                              SsBase + ((t + 1) & 1) * (BM + NBN));
      __syncthreads();
    }
  }
  if (do_cs && bn + (int)threadIdx.x < p.N) {
    const int64_t zo = EPI == CC_EPI_SPLITK ? (int64_t)split * p.N : 0;
    p.colsum[zo + bn + threadIdx.x] = cs;
  }

  // ---- epilogue: post-op fp32 tile -> LDS (passes of SR rows) -> coalesced stores
  float *S = reinterpret_cast<float *>(smem);  // [SR][SLD] (the K loop's buffers are done)
  float lossf = 0.f;
  const float scale = p.scale;
  float *Cf = p.Cf;
  int64_t ldf = p.ldc;
  if constexpr (EPI == CC_EPI_SPLITK) {
    Cf = p.Cf + (int64_t)split * p.M * p.N;
    ldf = p.N;
  }
  bf16_t *Cb = EPI == CC_EPI_SPLITK ? nullptr : reinterpret_cast<bf16_t *>(p.C);
  const bool vec = ((ldf & 3) == 0) && ((p.ldc & 3) == 0);
#pragma unroll 1
  for (int r0 = 0; r0 < BM; r0 += C::SR) {
    if (wm * 64 >= r0 && wm * 64 < r0 + C::SR) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int lc = wn * 64 + j * 32 + (lane & 31), gn = bn + lc;
          const int lr0 = wm * 64 + i * 32 + 4 * half;
          float bias = 0.f;
          if constexpr (EPI == CC_EPI_STORE || EPI == CC_EPI_BCE)
            bias = p.bias && gn < p.N ? p.bias[gn] : 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int lr = lr0 + (r & 3) + 8 * (r >> 2);
            float v = acc[i][j][r] + bias;
            if constexpr (EPI == CC_EPI_STORE) {
              if (p.relu) v = v > 0.f ? v : 0.f;
            } else if constexpr (EPI == CC_EPI_BCE && kBceRegs) {
              v = bce_dz(v, (ys[lr][lc >> 5] >> (lc & 31)) & 1u, scale, lossf,
                         bm + lr < p.M && gn < p.N);
            }
            S[(lr - r0) * SLD + lc] = v;        // BCE (!kBceRegs): the logit, transformed below
          }
        }
      }
    }
    __syncthreads();
    if constexpr (EPI == CC_EPI_BCE && kBceRegs) {
      if (r0 == 0) bce_publish(lossf);  // the loss is final after the register pass
    }
    if constexpr (EPI == CC_EPI_BCE && !kBceRegs) {
      // taller tiles: the transcendental work runs from LDS so it does not hold the
      // accumulators' registers (z -> dz in place)
      for (int idx = threadIdx.x; idx < C::SR * NBN; idx += NTH) {
        const int lr = idx / NBN, lc = idx % NBN;
        float &z = S[lr * SLD + lc];
        z = bce_dz(z, (ys[r0 + lr][lc >> 5] >> (lc & 31)) & 1u, scale, lossf,
                   bm + r0 + lr < p.M && bn + lc < p.N);
      }
      __syncthreads();
    }
    // rows of C / Cf: thread -> 4 consecutive columns
    for (int idx = threadIdx.x; idx < C::SR * (NBN / 4); idx += NTH) {
      const int lr = idx / (NBN / 4), lc = (idx % (NBN / 4)) * 4;
      const int gm = bm + r0 + lr, gn = bn + lc;
      if (gm >= p.M || gn >= p.N) continue;
      const float v0 = S[lr * SLD + lc], v1 = S[lr * SLD + lc + 1];
      const float v2 = S[lr * SLD + lc + 2], v3 = S[lr * SLD + lc + 3];
      if (vec && gn + 3 < p.N) {
        if (Cf) *reinterpret_cast<float4 *>(Cf + (int64_t)gm * ldf + gn) = make_float4(v0, v1, v2, v3);
        if (Cb) {
          const uint2 pk = make_uint2((uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16),
                                      (uint32_t)f2bf(v2) | ((uint32_t)f2bf(v3) << 16));
          *reinterpret_cast<uint2 *>(Cb + (int64_t)gm * p.ldc + gn) = pk;
        }
      } else {
        const float vv[4] = {v0, v1, v2, v3};
        for (int e = 0; e < 4 && gn + e < p.N; ++e) {
          if (Cf) Cf[(int64_t)gm * ldf + gn + e] = vv[e];
          if (Cb) Cb[(int64_t)gm * p.ldc + gn + e] = f2bf(vv[e]);
        }
      }
    }
    if constexpr (EPI == CC_EPI_BCE) {
      // rows of C^T [N][M] for this pass's rows: thread -> 8 consecutive m
      if (p.Ct) {
        bf16_t *Ct = reinterpret_cast<bf16_t *>(p.Ct);
        const bool vt = (p.ldct & 7) == 0;
        for (int idx = threadIdx.x; idx < NBN * (C::SR / 8); idx += NTH) {
          const int lc = idx / (C::SR / 8), lr = (idx % (C::SR / 8)) * 8;
          const int gn = bn + lc, gm = bm + r0 + lr;
          if (gn >= p.N || gm >= p.M) continue;
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = S[(lr + e) * SLD + lc];
          bf16_t *dst = Ct + (int64_t)gn * p.ldct + gm;
          if (vt && gm + 7 < p.M) {
            uint4 pk;
            pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            pk.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
            pk.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
            *reinterpret_cast<uint4 *>(dst) = pk;
          } else {
            for (int e = 0; e < 8 && gm + e < p.M; ++e) dst[e] = f2bf(v[e]);
          }
        }
      }
    }
    __syncthreads();
  }
  if constexpr (EPI == CC_EPI_BCE) {
    if constexpr (!kBceRegs) bce_publish(lossf);
    if (p.loss_out) {  // the last tile block reduces the partials in tile order: the loss, no
      __syncthreads();  // separate reduce launch
      if (lastflag) {
        double s2 = 0.0;
        for (int i = threadIdx.x; i < nblk; i += NTH)
          s2 += __hip_atomic_load(&p.loss_partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s2 += __shfl_xor(s2, off);
        if (lane == 0) red[wave] = s2;
        __syncthreads();
        if (threadIdx.x == 0) {
          double tot = 0.0;
          for (int w = 0; w < NTH / 64; ++w) tot += red[w];
          p.loss_out[0] = tot * p.loss_scale;
          __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

// Split-K launches: the (split, tile) pairs are dealt to the XCDs in contiguous split-major runs,
// so every tile of one K-split runs on one XCD and the split's A and B panels come from beyond
// L2 once per XCD (tile-only remapping pinned each tile to one XCD across all splits, so the
// panels shared by a split's tiles were fetched once per tile: 113 MB vs ~50 MB per dX product).
__device__ __forceinline__ void split_pair(int lin, int nb, int splits, int &tile, int &split) {
  const int q = xcd_tile(lin, nb * splits);
  split = q / nb;
  tile = q % nb;
}

template <int EPI, int BM>
__global__ __launch_bounds__(NtCfg<BM>::NTH) void gemm_nt_bf16_kernel(GemmParams p, int tiles_m) {
  __shared__ __attribute__((aligned(16))) char smem[NtCfg<BM>::LDS];
  __shared__ uint32_t ys[EPI == CC_EPI_BCE ? BM : 1][NBN / 32];  // BCE targets of the tile
  __shared__ double red[NtCfg<BM>::NTH / 64];
  __shared__ int lastflag;
  if constexpr (EPI == CC_EPI_SPLITK) {
    int tile, split;
    split_pair(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x, gridDim.y, tile, split);
    nt_body<EPI, BM>(p, tiles_m, tile, gridDim.x, split, smem, ys, red, lastflag, true);
  } else {
    nt_body<EPI, BM>(p, tiles_m, blockIdx.x, gridDim.x, blockIdx.y, smem, ys, red, lastflag);
  }
}

// The same tiles on MX-FP8 operands (128 x 128, K % 128 == 0).
template <int EPI>
__global__ __launch_bounds__(256) void gemm_nt_mx8_kernel(GemmParams p, int tiles_m) {
  __shared__ __attribute__((aligned(16))) char smem[NtCfg<128, uint8_t>::LDS];
  __shared__ uint32_t ys[EPI == CC_EPI_BCE ? 128 : 1][NBN / 32];
  __shared__ double red[NtCfg<128, uint8_t>::NTH / 64];
  __shared__ int lastflag;
  if constexpr (EPI == CC_EPI_SPLITK) {
    int tile, split;
    split_pair(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x, gridDim.y, tile, split);
    nt_body<EPI, 128, uint8_t>(p, tiles_m, tile, gridDim.x, split, smem, ys, red, lastflag, true);
  } else {
    nt_body<EPI, 128, uint8_t>(p, tiles_m, blockIdx.x, gridDim.x, blockIdx.y, smem, ys, red, lastflag);
  }
}

// Two independent NT problems in one launch (grouped GEMM): blocks [0, nb0*s0) are problem 0's
// (tile, split) pairs, the rest problem 1's — the decoder's dX (split-K) and dW products fill
// the chip together instead of one after the other.
template <int E0, int E1, typename T = bf16_t>
__global__ __launch_bounds__(256) void gemm_nt_pair_kernel(GemmParams p0, int tm0, int nb0,
                                                                          int s0, GemmParams p1, int tm1,
                                                                          int nb1) {
  static_assert(E0 != CC_EPI_BCE && E1 != CC_EPI_BCE, "pair: no loss hand-off");
  __shared__ __attribute__((aligned(16))) char smem[NtCfg<128, T>::LDS];
  __shared__ uint32_t ys[1][NBN / 32];
  __shared__ double red[NtCfg<128, T>::NTH / 64];
  __shared__ int lastflag;
  const int b = blockIdx.x;
  if (b < nb0 * s0) {
    if constexpr (E0 == CC_EPI_SPLITK) {
      int tile, split;
      split_pair(b, nb0, s0, tile, split);
      nt_body<E0, 128, T>(p0, tm0, tile, nb0, split, smem, ys, red, lastflag, true);
    } else {
      nt_body<E0, 128, T>(p0, tm0, b % nb0, nb0, b / nb0, smem, ys, red, lastflag);
    }
  } else {
    const int c = b - nb0 * s0;
    nt_body<E1, 128, T>(p1, tm1, c % nb1, nb1, c / nb1, smem, ys, red, lastflag);
  }
}

template <int EPI>
int launch_nt_mx8(const cc_gemm_args *g, const GemmParams &p, hipStream_t s) {
  const int tm = (int)cdiv(g->M, 128), tn = (int)cdiv(g->N, NBN);
  const dim3 grid((unsigned)(tm * tn), EPI == CC_EPI_SPLITK ? (unsigned)g->splits : 1u);
  hipLaunchKernelGGL((gemm_nt_mx8_kernel<EPI>), grid, dim3(NtCfg<128, uint8_t>::NTH), 0, s, p, tm);
  CC_LAUNCH_CHECK("gemm_nt_mx8_kernel");
  return CC_OK;
}

template <int EPI, int BM>
int launch_nt_bm(const cc_gemm_args *g, const GemmParams &p, hipStream_t s) {
  const int tm = (int)cdiv(g->M, BM), tn = (int)cdiv(g->N, NBN);
  const dim3 grid((unsigned)(tm * tn), EPI == CC_EPI_SPLITK ? (unsigned)g->splits : 1u);
  hipLaunchKernelGGL((gemm_nt_bf16_kernel<EPI, BM>), grid, dim3(NtCfg<BM>::NTH), 0, s, p, tm);
  CC_LAUNCH_CHECK("gemm_nt_bf16_kernel");
  return CC_OK;
}

// Tile height: 128 rows by default (taller tiles read each B panel fewer times but measured
// slower on the decoder shapes, tools/micro/gemm_bench.py); CCREC_NT_BM=256/512 selects them.
template <int EPI>
int launch_nt(const cc_gemm_args *g, const GemmParams &p, hipStream_t s) {
  constexpr int forced = CCREC_NT_BM;  // build knob for benchmarking tile heights (0: 128)
  int bm = 128;  // measured fastest for the decoder shapes (K = 256 / 512 / split V)
  if (forced == 128 || forced == 256 || forced == 512) bm = forced;
  if (bm == 512) return launch_nt_bm<EPI, 512>(g, p, s);
  if (bm == 256) return launch_nt_bm<EPI, 256>(g, p, s);
  return launch_nt_bm<EPI, 128>(g, p, s);
}

template <typename T, int EPI, int BK>
int launch_bk(const cc_gemm_args *g, const GemmParams &p, hipStream_t s) {
  const dim3 grid((unsigned)cdiv(g->N, BN), (unsigned)cdiv(g->M, BM),
                  EPI == CC_EPI_SPLITK ? (unsigned)g->splits : 1u);
  const dim3 block(NT);
  if (g->ta && g->tb)
    hipLaunchKernelGGL((gemm_kernel<T, true, true, EPI, BK>), grid, block, 0, s, p);
  else if (g->ta)
    hipLaunchKernelGGL((gemm_kernel<T, true, false, EPI, BK>), grid, block, 0, s, p);
  else if (g->tb)
    hipLaunchKernelGGL((gemm_kernel<T, false, true, EPI, BK>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_kernel<T, false, false, EPI, BK>), grid, block, 0, s, p);
  CC_LAUNCH_CHECK("gemm_kernel");
  return CC_OK;
}

// K-tile depth: a deeper BK puts more bytes in flight per iteration of the latency-bound K loop.
template <typename T, int EPI>
int launch_t(const cc_gemm_args *g, const GemmParams &p, hipStream_t s) {
  const int kc = EPI == CC_EPI_SPLITK ? (int)cdiv(g->K, g->splits) : g->K;
  if (sizeof(T) == 2 && kc >= 512) return launch_bk<T, EPI, 128>(g, p, s);
  if (kc >= 128) return launch_bk<T, EPI, 64>(g, p, s);
  return launch_bk<T, EPI, 32>(g, p, s);
}

template <typename T>
int launch_epi(const cc_gemm_args *g, const GemmParams &p, hipStream_t s) {
  switch (g->epilogue) {
    case CC_EPI_STORE: return launch_t<T, CC_EPI_STORE>(g, p, s);
    case CC_EPI_BCE: return launch_t<T, CC_EPI_BCE>(g, p, s);
    case CC_EPI_MASK: return launch_t<T, CC_EPI_MASK>(g, p, s);
    case CC_EPI_SPLITK: return launch_t<T, CC_EPI_SPLITK>(g, p, s);
  }
  return cc::fail(CC_ERR_ARG, "cc_gemm: unknown epilogue");
}

// ---------------------------------------------------------------- split-K reduce / colsum / loss
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float *__restrict__ part,
                                                            int splits, int M, int N,
                                                            const T *__restrict__ H, T *C,
                                                            float *Cf, const float *cs_part,
                                                            float *cs_out, const void *warm, int64_t warm_bytes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MN = (int64_t)M * N;
  l2_warm(warm, warm_bytes, blockIdx.x, gridDim.x);  // the next launch's operands (tower backward)
  if (cs_out && i < N) {
    float c = 0.f;
    for (int z = 0; z < splits; ++z) c += cs_part[(int64_t)z * N + i];
    cs_out[i] = c;
  }
  if (i >= MN) return;
  // the splits' loads are independent: issue 8 at a time, add in split order
  float s = 0.f;
  int z = 0;
  for (; z + 8 <= splits; z += 8) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = part[(int64_t)(z + u) * MN + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
  }
  for (; z < splits; ++z) s += part[(int64_t)z * MN + i];
  if (H) s = DT<T>::ld(H + i) > 0.f ? s : 0.f;
  if (C) DT<T>::st(C + i, s);
  if (Cf) Cf[i] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T *__restrict__ X, int R, int N, int ld,
                                                     float *__restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += DT<T>::ld(X + (int64_t)r * ld + n);
  out[n] = s;
}

// bf16 transpose with 16-B accesses on both sides (rows, cols multiples of 8, 16-B aligned):
// a 64 x 64 tile moves as 512 chunks of 8 elements in and 512 out (2 per thread).
__global__ __launch_bounds__(256) void transpose_b16v_kernel(const bf16_t *__restrict__ src, int rows,
                                                            int cols, bf16_t *__restrict__ dst) {
  __shared__ bf16_t tile[64][64 + 2];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  uint4 in[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + 256 * k, r = r0 + q / 8, c = c0 + (q % 8) * 8;
    in[k] = r < rows && c < cols ? *reinterpret_cast<const uint4 *>(src + (int64_t)r * cols + c)
                                 : make_uint4(0u, 0u, 0u, 0u);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + 256 * k, rr = q / 8, cc = (q % 8) * 8;
    const uint32_t w[4] = {in[k].x, in[k].y, in[k].z, in[k].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[rr][cc + 2 * e] = (bf16_t)(w[e] & 0xFFFFu);
      tile[rr][cc + 2 * e + 1] = (bf16_t)(w[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + 256 * k, cc = q / 8, rr = (q % 8) * 8;
    const int c = c0 + cc, r = r0 + rr;
    if (c >= cols || r >= rows) continue;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)tile[rr + 2 * e][cc] | ((uint32_t)tile[rr + 2 * e + 1][cc] << 16);
    *reinterpret_cast<uint4 *>(dst + (int64_t)c * rows + r) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T *__restrict__ src, int rows, int cols,
                                                        T *__restrict__ dst) {
  __shared__ T tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = r0 + e / 64, c = c0 + e % 64;
    if (r < rows && c < cols) tile[e / 64][e % 64] = src[(int64_t)r * cols + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int c = c0 + e / 64, r = r0 + e % 64;
    if (r < rows && c < cols) dst[(int64_t)c * rows + r] = tile[e % 64][e / 64];
  }
}

__global__ void reduce_loss_kernel(const double *__restrict__ part, int n, double scale,
                                   double *out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += part[i];
  const double t = block_sum_double(s, red);
  if (threadIdx.x == 0) out[0] = t * scale;
}

}  // namespace

extern "C" int cc_gemm_grid(int32_t M, int32_t N, int32_t *tiles) {
  CC_REQUIRE(tiles, "cc_gemm_grid: null");
  *tiles = (int32_t)(cdiv(M, BM) * cdiv(N, BN));
  return CC_OK;
}

static int gemm_params(const cc_gemm_args *g, GemmParams &p) {
  CC_REQUIRE(g && g->A && g->B, "cc_gemm: null operand");
  CC_REQUIRE(g->M >= 0 && g->N >= 0 && g->K >= 0, "cc_gemm: negative size");
  CC_REQUIRE(g->dtype == CC_BF16 || g->dtype == CC_F32 || g->dtype == CC_MX8, "cc_gemm: dtype");
  if (g->dtype == CC_MX8) {
    CC_REQUIRE(!g->ta && g->tb, "cc_gemm: MX8 is NT only (ta = 0, tb = 1)");
    CC_REQUIRE(g->K % 128 == 0 && g->lda % 128 == 0 && g->ldb % 128 == 0,
               "cc_gemm: MX8 needs K, lda, ldb multiples of 128");
    CC_REQUIRE(g->a_scale && g->b_scale && ((uintptr_t)g->a_scale | (uintptr_t)g->b_scale) % 4 == 0,
               "cc_gemm: MX8 needs 4-byte aligned a_scale / b_scale");
    CC_REQUIRE(((uintptr_t)g->A | (uintptr_t)g->B) % 16 == 0, "cc_gemm: MX8 operands 16-byte aligned");
    CC_REQUIRE(g->epilogue != CC_EPI_MASK && !g->colsum, "cc_gemm: MX8 epilogues STORE/BCE/SPLITK, no colsum");
  }
  if (g->epilogue == CC_EPI_SPLITK) CC_REQUIRE(g->splits >= 1 && g->Cf, "cc_gemm: split-K needs Cf, splits>=1");
  if (g->epilogue == CC_EPI_BCE)
    CC_REQUIRE(g->bias && g->y_bits && g->loss_partials, "cc_gemm: BCE needs bias, y_bits, loss_partials");
  if (g->epilogue == CC_EPI_MASK) CC_REQUIRE(g->H, "cc_gemm: MASK needs H");
  const int vw = g->dtype == CC_MX8 ? 16 : g->dtype == CC_BF16 ? 8 : 4;
  p.M = g->M; p.N = g->N; p.K = g->K;
  p.lda = g->lda; p.ldb = g->ldb; p.ldc = g->ldc;
  p.splits = g->splits; p.relu = g->relu;
  p.vec_a = (g->lda % vw == 0) && ((uintptr_t)g->A % 16 == 0);
  p.vec_b = (g->ldb % vw == 0) && ((uintptr_t)g->B % 16 == 0);
  p.A = g->A; p.B = g->B; p.bias = g->bias; p.C = g->C; p.Cf = g->Cf; p.H = g->H;
  p.y_bits = g->y_bits; p.scale = g->scale; p.loss_partials = g->loss_partials;
  p.colsum = g->colsum;
  p.Ct = g->Ct;
  p.ldct = g->ldct;
  p.loss_out = g->epilogue == CC_EPI_BCE ? g->loss_out : nullptr;
  p.loss_scale = g->loss_scale;
  p.ticket = g->ticket;
  p.sa = g->a_scale;
  p.sb = g->b_scale;
  CC_REQUIRE(!p.loss_out || p.ticket, "cc_gemm: loss_out needs a ticket word");
  CC_REQUIRE(!g->Ct || g->epilogue == CC_EPI_BCE, "cc_gemm: Ct only with the BCE epilogue");
  return CC_OK;
}

// bf16 with both operands K-contiguous and 16-B aligned rows: the 128x128 NT kernel
static bool nt_path(const cc_gemm_args *g, const GemmParams &p) {
  constexpr bool nt_enabled = CCREC_GEMM_NT;  // build knob for benchmarking the generic kernel
  return nt_enabled && g->dtype == CC_BF16 && !g->ta && g->tb && p.vec_a && p.vec_b &&
         g->epilogue != CC_EPI_MASK;
}

// MX-FP8 STORE / split-K / BCE products go to the 256 x 256 LDS-DMA kernel (mx8gemm.hip; bit-identical
// results); cc_gemm_tile128 keeps them on the 128 x 128 kernel (the reference of the bit-identity tests).
static bool mx8_wide_ok(const cc_gemm_args *g) {
  const bool bce_ok = g->epilogue == CC_EPI_BCE && g->C && (int64_t)g->M * g->ldc * 2 < 0x100000000ll &&
                      (!g->Ct || ((uintptr_t)g->Ct % 8 == 0 && g->ldct % 4 == 0 && g->M % 4 == 0 &&
                                  (int64_t)g->N * g->ldct * 2 < 0x80000000ll));
  return g->dtype == CC_MX8 && (g->epilogue == CC_EPI_STORE || g->epilogue == CC_EPI_SPLITK || bce_ok) &&
         g->M > 0 && g->N > 0 && !g->relu && !g->colsum && (!g->Ct || bce_ok) &&
         (int64_t)g->M * g->lda < 0x80000000ll && (int64_t)g->N * g->ldb < 0x80000000ll &&
         (g->epilogue == CC_EPI_SPLITK || g->ldc >= g->N);
}

static int gemm_dispatch(const cc_gemm_args *g, void *stream, bool wide) {
  GemmParams p;
  if (int rc = gemm_params(g, p)) return rc;
  if (g->M == 0 || g->N == 0) return CC_OK;
  hipStream_t s = as_stream(stream);
  if (wide && mx8_wide_ok(g)) return cc_gemm_mx8_wide(g, nullptr, stream);
  if (g->dtype == CC_MX8) {
    switch (g->epilogue) {
      case CC_EPI_STORE: return launch_nt_mx8<CC_EPI_STORE>(g, p, s);
      case CC_EPI_BCE: return launch_nt_mx8<CC_EPI_BCE>(g, p, s);
      case CC_EPI_SPLITK: return launch_nt_mx8<CC_EPI_SPLITK>(g, p, s);
    }
    return cc::fail(CC_ERR_ARG, "cc_gemm: MX8 epilogue");
  }
  if (nt_path(g, p)) {
    switch (g->epilogue) {
      case CC_EPI_STORE: return launch_nt<CC_EPI_STORE>(g, p, s);
      case CC_EPI_BCE: return launch_nt<CC_EPI_BCE>(g, p, s);  // reduces the loss itself
      case CC_EPI_SPLITK: return launch_nt<CC_EPI_SPLITK>(g, p, s);
    }
  }
  const double *lo = p.loss_out;
  p.loss_out = nullptr;  // the generic kernel writes partials only; reduce them after it
  const int rc = g->dtype == CC_BF16 ? launch_epi<bf16_t>(g, p, s) : launch_epi<float>(g, p, s);
  if (rc != CC_OK || !lo) return rc;
  int32_t tiles = 0;
  cc_gemm_grid(g->M, g->N, &tiles);
  return cc_reduce_loss(g->loss_partials, tiles, g->loss_scale, g->loss_out, stream);
}

extern "C" int cc_gemm(const cc_gemm_args *g, void *stream) { return gemm_dispatch(g, stream, true); }

extern "C" int cc_gemm_tile128(const cc_gemm_args *g, void *stream) { return gemm_dispatch(g, stream, false); }

extern "C" int cc_gemm_pair(const cc_gemm_args *g0, const cc_gemm_args *g1, void *stream) {
  GemmParams p0, p1;
  if (int rc = gemm_params(g0, p0)) return rc;
  if (int rc = gemm_params(g1, p1)) return rc;
  auto pairable = [](const cc_gemm_args *g, const GemmParams &p) {
    return (nt_path(g, p) || g->dtype == CC_MX8) && g->M > 0 && g->N > 0 &&
           (g->epilogue == CC_EPI_STORE || g->epilogue == CC_EPI_SPLITK);
  };
  if (mx8_wide_ok(g0) && mx8_wide_ok(g1)) return cc_gemm_mx8_wide(g0, g1, stream);
  if (!pairable(g0, p0) || !pairable(g1, p1) || (g0->dtype == CC_MX8) != (g1->dtype == CC_MX8)) {
    if (int rc = cc_gemm(g0, stream)) return rc;
    return cc_gemm(g1, stream);
  }
  const int tm0 = (int)cdiv(g0->M, 128), nb0 = tm0 * (int)cdiv(g0->N, NBN);
  const int tm1 = (int)cdiv(g1->M, 128), nb1 = tm1 * (int)cdiv(g1->N, NBN);
  const int s0 = g0->epilogue == CC_EPI_SPLITK ? g0->splits : 1;
  const int s1 = g1->epilogue == CC_EPI_SPLITK ? g1->splits : 1;
  const dim3 grid((unsigned)(nb0 * s0 + nb1 * s1)), block(NtCfg<128>::NTH);
  hipStream_t s = as_stream(stream);
#define PAIR(E0, E1)                                                                                     \
  do {                                                                                                   \
    if (g0->dtype == CC_MX8)                                                                             \
      hipLaunchKernelGGL((gemm_nt_pair_kernel<E0, E1, uint8_t>), grid, block, 0, s, p0, tm0, nb0, s0, p1, tm1, nb1); \
    else                                                                                                 \
      hipLaunchKernelGGL((gemm_nt_pair_kernel<E0, E1>), grid, block, 0, s, p0, tm0, nb0, s0, p1, tm1, nb1); \
  } while (0)
  if (g0->epilogue == CC_EPI_SPLITK && g1->epilogue == CC_EPI_STORE) PAIR(CC_EPI_SPLITK, CC_EPI_STORE);
  else if (g0->epilogue == CC_EPI_STORE && g1->epilogue == CC_EPI_SPLITK) PAIR(CC_EPI_STORE, CC_EPI_SPLITK);
  else if (g0->epilogue == CC_EPI_STORE) PAIR(CC_EPI_STORE, CC_EPI_STORE);
  else PAIR(CC_EPI_SPLITK, CC_EPI_SPLITK);
#undef PAIR
  CC_LAUNCH_CHECK("gemm_nt_pair_kernel");
  return CC_OK;
}

extern "C" int cc_splitk_reduce_warm(int32_t dtype, const float *partials, int32_t splits, int32_t M,
                                     int32_t N, const void *H, void *C, float *Cf,
                                     const float *colsum_partials, float *colsum_out, const void *warm,
                                     int64_t warm_bytes, void *stream);

extern "C" int cc_splitk_reduce(int32_t dtype, const float *partials, int32_t splits, int32_t M,
                                int32_t N, const void *H, void *C, float *Cf,
                                const float *colsum_partials, float *colsum_out, void *stream) {
  return cc_splitk_reduce_warm(dtype, partials, splits, M, N, H, C, Cf, colsum_partials, colsum_out,
                               nullptr, 0, stream);
}

extern "C" int cc_splitk_reduce_warm(int32_t dtype, const float *partials, int32_t splits, int32_t M,
                                     int32_t N, const void *H, void *C, float *Cf,
                                     const float *colsum_partials, float *colsum_out, const void *warm,
                                     int64_t warm_bytes, void *stream) {
  CC_REQUIRE(partials && splits >= 1, "cc_splitk_reduce: args");
  const int64_t MN = (int64_t)M * N;
  if (MN == 0) return CC_OK;
  const dim3 grid((unsigned)cdiv(MN, 256)), block(256);
  if (dtype == CC_BF16)
    hipLaunchKernelGGL(splitk_reduce_kernel<bf16_t>, grid, block, 0, as_stream(stream), partials,
                       splits, M, N, (const bf16_t *)H, (bf16_t *)C, Cf, colsum_partials, colsum_out,
                       warm, warm_bytes);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, grid, block, 0, as_stream(stream), partials,
                       splits, M, N, (const float *)H, (float *)C, Cf, colsum_partials, colsum_out,
                       warm, warm_bytes);
  CC_LAUNCH_CHECK("splitk_reduce_kernel");
  return CC_OK;
}

extern "C" int cc_colsum(int32_t dtype, const void *X, int32_t R, int32_t N, int32_t ld,
                         float *out, void *stream) {
  CC_REQUIRE(X && out, "cc_colsum: null");
  if (N == 0) return CC_OK;
  const dim3 grid((unsigned)cdiv(N, 256)), block(256);
  if (dtype == CC_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, block, 0, as_stream(stream), (const bf16_t *)X, R, N, ld, out);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, block, 0, as_stream(stream), (const float *)X, R, N, ld, out);
  CC_LAUNCH_CHECK("colsum_kernel");
  return CC_OK;
}

extern "C" int cc_transpose(int32_t dtype, const void *src, int32_t rows, int32_t cols, void *dst,
                            void *stream) {
  CC_REQUIRE(src && dst && rows >= 0 && cols >= 0, "cc_transpose: args");
  if (rows == 0 || cols == 0) return CC_OK;
  const dim3 grid((unsigned)cdiv(cols, 64), (unsigned)cdiv(rows, 64)), block(256);
  if (dtype == CC_BF16 && rows % 8 == 0 && cols % 8 == 0 && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0) {
    hipLaunchKernelGGL(transpose_b16v_kernel, grid, block, 0, as_stream(stream), (const bf16_t *)src,
                       rows, cols, (bf16_t *)dst);
    CC_LAUNCH_CHECK("transpose_b16v_kernel");
    return CC_OK;
  }
  if (dtype == CC_BF16)
    hipLaunchKernelGGL(transpose_kernel<bf16_t>, grid, block, 0, as_stream(stream), (const bf16_t *)src, rows, cols, (bf16_t *)dst);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, block, 0, as_stream(stream), (const float *)src, rows, cols, (float *)dst);
  CC_LAUNCH_CHECK("transpose_kernel");
  return CC_OK;
}

extern "C" int cc_reduce_loss(const double *partials, int32_t n, double scale, double *loss_out,
                              void *stream) {
  CC_REQUIRE(partials && loss_out && n >= 0, "cc_reduce_loss: args");
  hipLaunchKernelGGL(reduce_loss_kernel, dim3(1), dim3(256), 0, as_stream(stream), partials, n,
                     scale, loss_out);
  CC_LAUNCH_CHECK("reduce_loss_kernel");
  return CC_OK;
}

extern "C" int cc_dec_bce_fused(int32_t dtype, const void *H3, const void *Wo, const float *bo,
                                int32_t B, int32_t d, int32_t V, const uint32_t *y_bits, void *dZ,
                                double *loss_partials, int32_t *n_partials, void *stream) {
  cc_gemm_args g = {};
  g.dtype = dtype; g.ta = 0; g.tb = 0; g.epilogue = CC_EPI_BCE;
  g.M = B; g.N = V; g.K = d; g.lda = d; g.ldb = V; g.ldc = V;
  g.A = H3; g.B = Wo; g.bias = bo; g.C = dZ; g.y_bits = y_bits;
  g.scale = 1.0f / ((float)B * (float)V);
  g.loss_partials = loss_partials;
  if (n_partials) *n_partials = (int32_t)(cdiv(B, BM) * cdiv(V, BN));
  return cc_gemm(&g, stream);
}
