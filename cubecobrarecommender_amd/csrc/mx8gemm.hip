// MX-FP8 NT GEMM on 256 x 256 tiles with an LDS-DMA stage pipeline — config 5's decoder output
// layer products (model.py:64 Dense(V) at d = 1024 and its backward, the regulariser's logits
// model.py:98): C[M][N] = A[M][K] . B[N][K]^T, both operands e4m3 codes K-contiguous with one E8M0
// scale per 32 K (cc_quant_mx8), v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulation.
//
// Why a second kernel next to gemm.hip's 128 x 128 register-staged NT kernel: at d = 1024 that
// kernel reaches ~0.58 PFLOP/s (12 % of the MX-FP8 peak, tools/micro/mx8_bench.py) — a 128 x 128
// tile with 2 x 2 accumulators per wave reads 2 KB of LDS per MFMA, its register staging leaves
// few tiles in flight, and the decoder shapes have only 4-8 K-tiles per output tile.  Here:
//   * 8 waves as 2 (M) x 4 (N); a wave owns 128 x 64 outputs = 4 x 2 accumulators of 32 x 32, so
//     its 6 fragments per 64-k step feed 8 MFMAs (1.5 KB of LDS per MFMA);
//   * a K-tile is 128 fp8 of every row: A 256 x 128 B + B 256 x 128 B + the 4 scale bytes of each
//     row, copied global -> LDS by buffer_load ... lds (16-B chunks, 8 rows x 128 B per wave
//     instruction; scale words 4 B per lane), two stages: tile t + 1's DMA runs under tile t's
//     MFMAs.  The LDS images are lane-linear; the 16-B chunk swizzle (chunk ^ (row >> 1 & 7)) is applied
//     on the global source address, so fragment reads are the conflict-free pattern of gemm.hip's
//     nt_frag8.  Rows past M / N read zeros (their outputs are not stored);
//   * (tile, split) pairs are dealt to the XCDs in contiguous runs (tiles sharing a B panel, or a
//     K split's panels, run on one XCD and fetch the panel into its L2 once).
// The MFMA sequence of every output (k-tiles ascending, two 64-k steps each) is the one gemm.hip's
// MX kernel runs, so the results are bit-identical to it (tests/test_gpu_kernels.py).
// Epilogues: STORE (optional bias; fp32 Cf and/or bf16 C), SPLITK (fp32 partials [split][M][N]) and
// BCE (logits + bias -> sigmoid / BCE: dZ rows and optionally dZ^T in bf16, per-tile loss partials
// reduced in tile order by the last block when loss_out is set).
#include <cstdlib>

#include "common.hpp"
#include "mx8.hpp"

namespace {

// MX8_QNS (build knob): 2 = K tiles of 128 in two LDS stages (one tile of lead); 4 = K tiles of 64
// (one 32x32x64 step) in four stages, three tiles in flight while the fourth is multiplied.  Split-K
// chunks stay multiples of 128 either way (the same partition, the same bits).
#ifndef MX8_QNS
#define MX8_QNS 2
#endif
constexpr int QNS = MX8_QNS;
static_assert(QNS == 2 || QNS == 4, "MX8_QNS: 2 or 4");
constexpr int QM = 256, QN = 256, QKB = QNS == 2 ? 128 : 64, QNT = 512;
constexpr int QA_BYTES = QM * QKB, QB_BYTES = QN * QKB;
constexpr int QSTAGE = QA_BYTES + QB_BYTES + (QM + QN) * 4;   // + each row's E8M0 word of the 128 k
constexpr int QLDS = QNS * QSTAGE;  // 132 KB
// the BCE epilogue's LDS: a 256 x 130 fp32 pass tile, the 256 x 8 target words, the loss reduction
constexpr int QLDS_BCE = QM * 130 * 4 + QM * 8 * 4 + 8 * 8 + 16;
constexpr int QLDS_MAX = QLDS > QLDS_BCE ? QLDS : QLDS_BCE;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
// the stage copies as inline asm (M0 = the wave-uniform LDS address): the compiler does not count
// them, so it inserts no vmcnt before the fragment reads (LDS-DMA alias tracking would drain the
// copies in flight); q_body's waits are explicit
__device__ __forceinline__ i32x4_t q_rsrc(const void *base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  return i32x4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)a), __builtin_amdgcn_readfirstlane((int)(a >> 32) & 0xFFFF),
                 __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
__device__ __forceinline__ uint32_t q_lds(const void *p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_void *)p);
}
__device__ __forceinline__ void q_dma16(const i32x4_t &rs, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(lds) : "memory");
}
__device__ __forceinline__ void q_dma4(const i32x4_t &rs, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(lds) : "memory");
}
typedef __attribute__((ext_vector_type(8))) int i32x8_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

struct QP {
  const uint8_t *A, *B, *sa, *sb;
  const float *bias;
  bf16_t *C;
  float *Cf;
  // BCE epilogue (model.py:94 sigmoid + train.py:85 binary_crossentropy on the logits)
  const uint32_t *y_bits;  // [M][ceil(N/32)] targets
  bf16_t *Ct;              // optional dZ^T [N][ldct]
  double *loss_partials;   // [ntiles]
  double *loss_out;        // optional: the last block reduces the partials in tile order
  uint32_t *ticket;
  double loss_scale;
  float scale;
  int ldct;
  // optional MX-FP8 images of the bf16-rounded dZ, exactly as cc_quant_mx8 makes them from dZ:
  // zq [M][ldzq] (K = N; columns [N, ldzq) zero codes) + zqs [M][ldzq/32], ztq [N][ldztq] (K = M)
  // + ztqs [N][ldztq/32]; colsum[N] += the tile's column sums of the bf16 dZ (the bias gradient)
  uint8_t *zq, *zqs, *ztq, *ztqs;
  float *colsum;
  int ldzq, ldztq;
  int M, N, K, lda, ldb, ldc, splits, kchunk, tiles_m, ntiles, epi;
  uint32_t a_bytes, b_bytes, sa_bytes, sb_bytes;
};

// sigmoid_cross_entropy_with_logits (TF 2.5 Keras BCE on a sigmoid output):
//   loss = max(z, 0) - z y + log1p(exp(-|z|)),  dz = (sigmoid(z) - y) * scale,
// from a = exp(-|z|) by the hardware exp2 / rcp (decout.hip's forms).  The log1p terms of a lane's
// 16 rows are taken as ONE log2 of the product of their 1 + a in (1, 2] (<= 2^16; decout.hip):
// `lprod` collects the factors, `rsum` the max(+-z, 0) parts; dead elements contribute 1 and 0
__device__ __forceinline__ float q_bce(float z, uint32_t ybit, float scale, float &lprod, float &rsum, bool live) {
  constexpr float LOG2E = 1.4426950408889634f;
  const float a = __builtin_amdgcn_exp2f(-fabsf(z) * LOG2E);
  const float opa = 1.f + a;
  const float rp = __builtin_amdgcn_rcpf(opa);
  lprod *= live ? opa : 1.f;
  rsum += live ? fmaxf(ybit ? -z : z, 0.f) : 0.f;
  const float sig = z >= 0.f ? rp : a * rp;
  return (sig - (float)ybit) * scale;
}

// cross-lane steps of the epilogue's MX block reductions as DPP moves (no LDS round trip, unlike
// __shfl_xor's ds_bpermute): lane ^ 1, lane ^ 2 (quad_perm) and the mirror inside 8 lanes (after the
// two quad steps every lane of a quad holds the quad's value, so the mirror pairs the two quads)
__device__ __forceinline__ float dpp_f(float v, int ctrl_sel) {
  const int x = __builtin_bit_cast(int, v);
  int y;
  if (ctrl_sel == 0) y = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);       // quad_perm [1,0,3,2]
  else if (ctrl_sel == 1) y = __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  else y = __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);                    // row_half_mirror
  return __builtin_bit_cast(float, y);
}

__device__ __forceinline__ int xcd_run(int b, int nb) {  // bijective: block -> XCD-contiguous id
  const int q = nb / 8, r = nb % 8, x = b % 8, slot = b / 8;
  return x < r ? x * (q + 1) + slot : r * (q + 1) + (x - r) * q + slot;
}

// stage st <- K-tile at k0 (64 k): wave w moves A rows [32w, 32w + 32) and B rows [32w, 32w + 32)
// (2 + 2 instructions of 16 rows x 64 B, the 16-B chunk swizzle chunk ^ (row >> 2 & 3) applied on
// the global source address), and one 4-B-per-lane instruction of scale words (the 4 E8M0 bytes of
// the 128 k holding the tile: its 2 are picked by the tile's parity): waves 0-3 the A rows
// [64w, 64w + 64), waves 4-7 the B rows: 5 DMA instructions per wave per tile
// (QKB = 128: 4 + 4 instructions of 8 rows x 128 B, swizzle chunk ^ row & 7; 9 per wave per tile)
constexpr int QNI = QA_BYTES / 1024 / 8;        // A (and B) instructions per wave per tile
constexpr int QDMA_PER_TILE = 2 * QNI + 1;
constexpr int QRPI = 1024 / QKB;                // rows per instruction
// (128-B rows: row >> 1 & 7 — see dxgemm.hip: under row & 7 the rows r and r + 8 of a ds_read_b128
// lane group share a bank slot)
__device__ __forceinline__ int q_swz(int row) { return QKB == 128 ? ((row >> 1) & 7) : ((row >> 2) & 3); }
__device__ __forceinline__ void q_dma(const QP &p, const i32x4_t &ra, const i32x4_t &rb, const i32x4_t &rsa,
                                      const i32x4_t &rsb, char *smem, int st, int bm, int bn, int k0) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  char *sA = smem + st * QSTAGE, *sB = sA + QA_BYTES, *sS = sB + QB_BYTES;
#pragma unroll
  for (int u = 0; u < QNI; ++u) {
    const int i = w * QNI + u;  // rows QRPI i .. QRPI (i + 1) - 1
    const int row = QRPI * i + lane / (QKB / 16);
    const int c = (lane % (QKB / 16)) ^ q_swz(row);
    const uint32_t oa = bm + row < p.M ? (uint32_t)(bm + row) * (uint32_t)p.lda + (uint32_t)(k0 + 16 * c) : 0x80000000u;
    const uint32_t ob = bn + row < p.N ? (uint32_t)(bn + row) * (uint32_t)p.ldb + (uint32_t)(k0 + 16 * c) : 0x80000000u;
    q_dma16(ra, oa, q_lds(sA + i * 1024));
    q_dma16(rb, ob, q_lds(sB + i * 1024));
  }
  const int row = (w & 3) * 64 + lane;
  if (w < 4) {
    const uint32_t os = bm + row < p.M ? (uint32_t)(bm + row) * (uint32_t)(p.lda / 32) + (uint32_t)(k0 / 128 * 4) : 0x80000000u;
    q_dma4(rsa, os, q_lds(sS + (w & 3) * 256));
  } else {
    const uint32_t os = bn + row < p.N ? (uint32_t)(bn + row) * (uint32_t)(p.ldb / 32) + (uint32_t)(k0 / 128 * 4) : 0x80000000u;
    q_dma4(rsb, os, q_lds(sS + QM * 4 + (w & 3) * 256));
  }
}

// the 32 x 64 fp8 fragment of rows `row` (lane & 31) for 64-k step kk: lane half h holds k 16h ..
// 16h + 15 (low 16 B) and 32 + 16h .. (high 16 B) — chunks 4kk + h and 4kk + 2 + h (gemm.hip
// nt_frag8), under the stage's chunk swizzle (64-B rows: row >> 2 & 3 puts 16 consecutive rows on
// 16 distinct 16-B bank groups)
__device__ __forceinline__ i32x8_t q_frag(const char *S, int row, int c0) {
  const i32x4_t lo = *reinterpret_cast<const i32x4_t *>(S + row * QKB + ((c0 ^ q_swz(row)) << 4));
  const i32x4_t hi = *reinterpret_cast<const i32x4_t *>(S + row * QKB + (((c0 + 2) ^ q_swz(row)) << 4));
  return i32x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <bool BCE>
__device__ __forceinline__ void q_body(const QP &p, int q, char *smem) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5;
  const int wm = w >> 2, wn = w & 3;
  const int split = q / p.ntiles, tile = q % p.ntiles;
  const int bm = (tile % p.tiles_m) * QM, bn = (tile / p.tiles_m) * QN;
  const int kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
  const int nk = kbeg < kend ? (kend - kbeg) / QKB : 0;  // K % 128 == 0 and kchunk % 128 == 0
  const i32x4_t ra = q_rsrc(p.A, p.a_bytes), rb = q_rsrc(p.B, p.b_bytes);
  const i32x4_t rsa = q_rsrc(p.sa, p.sa_bytes), rsb = q_rsrc(p.sb, p.sb_bytes);
  f32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // BCE: the tile's target words (256 rows x 8 words), 4 per thread, in flight during the K loop
  // (issued before the stage copies: older than every copy the loop waits for)
  constexpr bool bce = BCE;
  const int YW = (p.N + 31) >> 5;
  uint32_t yv[4] = {0u, 0u, 0u, 0u};
  if constexpr (bce) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = threadIdx.x + QNT * u, r = i >> 3, gw = (bn >> 5) + (i & 7);
      yv[u] = bm + r < p.M && gw < YW ? p.y_bits[(int64_t)(bm + r) * YW + gw] : 0u;
    }
  }
  const int ar = wm * 128 + (lane & 31), br = wn * 64 + (lane & 31);
#pragma unroll
  for (int s = 0; s < QNS - 1; ++s)
    if (s < nk) q_dma(p, ra, rb, rsa, rsb, smem, s, bm, bn, kbeg + s * QKB);
  for (int t = 0; t < nk; ++t) {
    // tile t landed in every wave (own copies counted: those of the tiles after t, up to QNS - 2 of
    // them, may stay in flight; then the barrier), and every wave finished reading the stage the
    // copy below overwrites (tile t - 1's: its LDS reads retired before the barrier)
    const int younger = min(QNS - 2, nk - 1 - t);
    if (younger >= 2)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * QDMA_PER_TILE) : "memory");
    else if (younger == 1)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(QDMA_PER_TILE) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + QNS - 1 < nk) q_dma(p, ra, rb, rsa, rsb, smem, (t + QNS - 1) % QNS, bm, bn, kbeg + (t + QNS - 1) * QKB);
    const char *sA = smem + (t % QNS) * QSTAGE, *sB = sA + QA_BYTES;
    const uint32_t *sS = reinterpret_cast<const uint32_t *>(sB + QB_BYTES);
    uint32_t wa[4], wb[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) wa[i] = sS[ar + 32 * i];
#pragma unroll
    for (int j = 0; j < 2; ++j) wb[j] = sS[QM + br + 32 * j];
#pragma unroll
    for (int kk = 0; kk < QKB / 64; ++kk) {
      // (QKB = 64: kbeg % 128 == 0, so t's parity places the tile's 64 k in the scale word's 128)
      const int c0 = 4 * kk + half, sh = QKB == 128 ? 8 * (2 * kk + half) : 8 * (2 * (t & 1) + half);
      i32x8_t b[2];
      int sb[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        b[j] = q_frag(sB, br + 32 * j, c0);
        sb[j] = (int)((wb[j] >> sh) & 0xFFu);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const i32x8_t a = q_frag(sA, ar + 32 * i, c0);
        const int sa = (int)((wa[i] >> sh) & 0xFFu);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b[j], acc[i][j], 0, 0, 0, sa, 0, sb[j]);
      }
    }
  }
  // ---- epilogue straight from the accumulators: lanes 0..31 of a half = 32 consecutive columns
  // of one row (128 B of fp32 per row per instruction)
  if (p.epi == CC_EPI_SPLITK) {
    float *out = p.Cf + (int64_t)split * p.M * p.N;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = bn + wn * 64 + j * 32 + (lane & 31);
      if (col >= p.N) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = bm + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          if (row < p.M) out[(int64_t)row * p.N + col] = acc[i][j][r];
        }
    }
    return;
  }
  if constexpr (bce) {
    // The epilogue runs from LDS, in two passes of 128 columns (the waves' j = 0 accumulators,
    // then j = 1): the fp32 logits of the pass S[256][QSP] (pitch 130: the column reads of the
    // dZ^T loop hit distinct banks) and the tile's target words ys[cb][row].  Transforming the
    // 128 accumulators in registers instead spilled (the fully unrolled BCE math of 128 values).
    constexpr int QSP = 130;
    float *S = reinterpret_cast<float *>(smem);
    uint32_t *ys = reinterpret_cast<uint32_t *>(smem + QM * QSP * 4);
    double *red = reinterpret_cast<double *>(smem + QM * QSP * 4 + QM * 8 * 4);
    int *lastflag = reinterpret_cast<int *>(smem + QM * QSP * 4 + QM * 8 * 4 + 8 * sizeof(double));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();   // every wave left the K loop: the stage buffers are free
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // column-block-major: ys[cb][row]
      const int i = threadIdx.x + QNT * u;
      ys[(i & 7) * QM + (i >> 3)] = yv[u];
    }
    float lossf = 0.f;
    const float scale = p.scale;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      // local column c in [0, 128) <-> global bn + (c / 32) * 64 + jp * 32 + c % 32
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          S[(wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half) * QSP + wn * 32 + (lane & 31)] = acc[i][jp][r];
      __syncthreads();
      // rows: thread -> 4 consecutive columns c (fixed per thread) of rows tid / 32 + 16 k; dz
      // replaces z in S.  The 8 lanes of a 32-column block are consecutive (one MX scale).
      {
        const int cq = threadIdx.x & 31, c = cq * 4;
        const int gc = bn + (c >> 5) * 64 + jp * 32 + (c & 31);
        const int cb = (gc - bn) >> 5;
        float bias4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) bias4[e] = gc + e < p.N ? p.bias[gc + e] : 0.f;
#pragma unroll 2
        for (int lr = threadIdx.x >> 5; lr < QM; lr += QNT / 32) {
          const int row = bm + lr;
          const uint32_t yw = ys[cb * QM + lr] >> (c & 31);
          const float2 z01 = *reinterpret_cast<const float2 *>(S + lr * QSP + c);
          const float2 z23 = *reinterpret_cast<const float2 *>(S + lr * QSP + c + 2);
          const float zz[4] = {z01.x, z01.y, z23.x, z23.y};
          float lprod = 1.f, rsum = 0.f, dz[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool live = row < p.M && gc + e < p.N;
            dz[e] = live ? q_bce(zz[e] + bias4[e], (yw >> e) & 1u, scale, lprod, rsum, true) : 0.f;
          }
          *reinterpret_cast<float2 *>(S + lr * QSP + c) = make_float2(dz[0], dz[1]);
          *reinterpret_cast<float2 *>(S + lr * QSP + c + 2) = make_float2(dz[2], dz[3]);
          lossf += rsum + __builtin_amdgcn_logf(lprod) * 0.6931471805599453f;
          if (p.C && row < p.M) {
            bf16_t *dst = p.C + (int64_t)row * p.ldc + gc;
            if (gc + 3 < p.N && (p.ldc & 3) == 0) {
              *reinterpret_cast<uint2 *>(dst) = make_uint2((uint32_t)f2bf(dz[0]) | ((uint32_t)f2bf(dz[1]) << 16),
                                                           (uint32_t)f2bf(dz[2]) | ((uint32_t)f2bf(dz[3]) << 16));
            } else {
              for (int e = 0; e < 4 && gc + e < p.N; ++e) dst[e] = f2bf(dz[e]);
            }
          }
          if (p.zq) {   // MX-FP8 rows (K = N)
            float v[4], amax = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = bf2f(f2bf(dz[e]));   // dead elements are exact zeros
              amax = fmaxf(amax, fabsf(v[e]));
            }
            amax = fmaxf(amax, dpp_f(amax, 0));
            amax = fmaxf(amax, dpp_f(amax, 1));
            amax = fmaxf(amax, dpp_f(amax, 2));
            const int ex = cc_mx8::block_exp(amax);
            int word = 0;
            word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[0], -ex), ldexpf(v[1], -ex), word, false);
            word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[2], -ex), ldexpf(v[3], -ex), word, true);
            if (row < p.M && gc < p.ldzq) {
              *reinterpret_cast<uint32_t *>(p.zq + (int64_t)row * p.ldzq + gc) = (uint32_t)word;
              if ((cq & 7) == 0) p.zqs[(int64_t)row * (p.ldzq / 32) + gc / 32] = (uint8_t)(ex + 127);
            }
          }
        }
      }
      if (p.Ct || p.ztq) {
        // columns: lane -> (column cc = lane / 4 of the wave's 16, rows 8 (lane & 3) .. + 8 of a
        // 32-row block); wave w takes columns 16 w .. + 16, the loop walks the 8 row blocks.  Pitch
        // 130: the 64 lanes' reads of one row offset hit 64 distinct banks.  The 4 lanes of a column
        // share the block's MX scale; the column sum runs over the blocks in the thread, then the 4 lanes
        __syncthreads();
        const int c = w * 16 + (lane >> 2), rc = lane & 3;
        const int gc = bn + (c >> 5) * 64 + jp * 32 + (c & 31);
        const bool cok = gc < p.N;
        float csum = 0.f;
#pragma unroll 2
        for (int rb = 0; rb < QM / 32; ++rb) {
          const int lr = rb * 32 + rc * 8, row = bm + lr;
          uint32_t pk[4];
          float v[8], amax = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bf16_t h0 = f2bf(S[(lr + 2 * e) * QSP + c]), h1 = f2bf(S[(lr + 2 * e + 1) * QSP + c]);
            pk[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
            v[2 * e] = bf2f(h0);   // rows past M hold dz = 0
            v[2 * e + 1] = bf2f(h1);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            amax = fmaxf(amax, fabsf(v[e]));
            csum += v[e];
          }
          if (p.Ct && cok && row < p.M) {
            bf16_t *dst = p.Ct + (int64_t)gc * p.ldct + row;
            if (row + 7 < p.M && (p.ldct & 7) == 0) {
              *reinterpret_cast<uint4 *>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            } else {
              for (int e = 0; e < 8 && row + e < p.M; ++e) dst[e] = (bf16_t)(pk[e >> 1] >> (16 * (e & 1)));
            }
          }
          if (p.ztq) {
            amax = fmaxf(amax, dpp_f(amax, 0));
            amax = fmaxf(amax, dpp_f(amax, 1));
            const int ex = cc_mx8::block_exp(amax);
            int w0 = 0, w1 = 0;
            w0 = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[0], -ex), ldexpf(v[1], -ex), w0, false);
            w0 = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[2], -ex), ldexpf(v[3], -ex), w0, true);
            w1 = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4], -ex), ldexpf(v[5], -ex), w1, false);
            w1 = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[6], -ex), ldexpf(v[7], -ex), w1, true);
            if (cok && row < p.M) {
              *reinterpret_cast<uint2 *>(p.ztq + (int64_t)gc * p.ldztq + row) = make_uint2((uint32_t)w0, (uint32_t)w1);
              if (rc == 0) p.ztqs[(int64_t)gc * (p.ldztq / 32) + row / 32] = (uint8_t)(ex + 127);
            }
          }
        }
        if (p.colsum) {
          csum += dpp_f(csum, 0);
          csum += dpp_f(csum, 1);
          // one row tile: stored; two (checked on the host): added onto the zeros of
          // colsum_zero_kernel, fl(fl(0 + a) + b) == fl(fl(0 + b) + a)
          if (cok && rc == 0) {
            if (p.tiles_m == 1)
              p.colsum[gc] = csum;
            else
              atomicAdd(p.colsum + gc, csum);
          }
        }
      }
      __syncthreads();   // S is rewritten by the next pass
    }
    // the tile's loss partial (waves in order), then the last tile block reduces them in tile order
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) lossf += __shfl_xor(lossf, off);
    if (lane == 0) red[w] = (double)lossf;
    __syncthreads();
    if (threadIdx.x == 0) {
      double sum = 0.0;
      for (int v = 0; v < QNT / 64; ++v) sum += red[v];
      *lastflag = 0;
      if (!p.loss_out) {
        p.loss_partials[tile] = sum;
      } else {
        __hip_atomic_store(&p.loss_partials[tile], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t tk = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lastflag = tk == (uint32_t)p.ntiles - 1;
      }
    }
    if (!p.loss_out) return;
    __syncthreads();
    if (!*lastflag) return;
    double s2 = 0.0;
    for (int v = threadIdx.x; v < p.ntiles; v += QNT)
      s2 += __hip_atomic_load(&p.loss_partials[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s2 += __shfl_xor(s2, off);
    __syncthreads();
    if (lane == 0) red[w] = s2;
    __syncthreads();
    if (threadIdx.x == 0) {
      double tot = 0.0;
      for (int v = 0; v < QNT / 64; ++v) tot += red[v];
      p.loss_out[0] = tot * p.loss_scale;
      __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = bn + wn * 64 + j * 32 + (lane & 31);
    if (col >= p.N) continue;
    const float bias = p.bias ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = bm + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (row >= p.M) continue;
        const float v = acc[i][j][r] + bias;
        if (p.Cf) p.Cf[(int64_t)row * p.ldc + col] = v;
        if (p.C) p.C[(int64_t)row * p.ldc + col] = f2bf(v);
      }
  }
}

template <bool BCE>
__global__ __launch_bounds__(QNT) void mx8_wide_kernel(QP p) {
  extern __shared__ __attribute__((aligned(1024))) char qsmem[];
  q_body<BCE>(p, xcd_run(blockIdx.x, p.ntiles * p.splits), qsmem);
}

// two independent problems in one launch (the decoder's dX split-K and dW products): blocks
// [0, n0) are problem 0's, the rest problem 1's, each dealt to the XCDs in contiguous runs
__global__ __launch_bounds__(QNT) void mx8_wide_pair_kernel(QP p0, QP p1) {
  extern __shared__ __attribute__((aligned(1024))) char qsmem[];
  const int n0 = p0.ntiles * p0.splits;
  if ((int)blockIdx.x < n0)
    q_body<false>(p0, xcd_run(blockIdx.x, n0), qsmem);
  else
    q_body<false>(p1, xcd_run(blockIdx.x - n0, p1.ntiles * p1.splits), qsmem);
}

// the BCE product with dZ's MX-FP8 images (problem 0, the first n0 blocks) and an independent
// STORE product (problem 1: config 5's regulariser logits, which read the same D3 launch's other
// rows) in one launch: 172 + 172 tiles at B = 512, |V| = 22,000 fill the 256 CUs that either
// alone leaves a third idle
__global__ __launch_bounds__(QNT) void mx8_bce_pair_kernel(QP p0, QP p1) {
  extern __shared__ __attribute__((aligned(1024))) char qsmem[];
  const int n0 = p0.ntiles;
  if ((int)blockIdx.x < n0)
    q_body<true>(p0, xcd_run(blockIdx.x, n0), qsmem);
  else
    q_body<false>(p1, xcd_run(blockIdx.x - n0, p1.ntiles * p1.splits), qsmem);
}

int q_params(const cc_gemm_args *g, QP &p) {
  CC_REQUIRE(g && g->dtype == CC_MX8 && !g->ta && g->tb, "cc_gemm_mx8_wide: MX8 NT only");
  CC_REQUIRE(g->A && g->B && g->a_scale && g->b_scale, "cc_gemm_mx8_wide: null operand");
  CC_REQUIRE(g->M > 0 && g->N > 0 && g->K > 0, "cc_gemm_mx8_wide: empty problem");
  CC_REQUIRE(g->K % 128 == 0 && g->lda % 128 == 0 && g->ldb % 128 == 0 && g->lda >= g->K && g->ldb >= g->K,
             "cc_gemm_mx8_wide: K, lda, ldb multiples of 128, lda / ldb >= K");
  CC_REQUIRE(g->epilogue == CC_EPI_STORE || g->epilogue == CC_EPI_SPLITK || g->epilogue == CC_EPI_BCE,
             "cc_gemm_mx8_wide: STORE, SPLITK or BCE");
  CC_REQUIRE(g->epilogue != CC_EPI_BCE || (g->bias && g->y_bits && g->loss_partials && g->C && g->ldc >= g->N &&
                                           (!g->Ct || g->ldct >= g->M) && (!g->loss_out || g->ticket)),
             "cc_gemm_mx8_wide: BCE needs bias, y_bits, loss_partials, C (ldc >= N), ldct >= M, a ticket with loss_out");
  CC_REQUIRE(!g->Ct || ((uintptr_t)g->Ct % 8 == 0 && g->ldct % 4 == 0 && g->M % 4 == 0 &&
                         (int64_t)g->N * g->ldct * 2 < 0x80000000ll),
             "cc_gemm_mx8_wide: Ct 8-B aligned rows, M % 4 == 0, below 2 GB");
  CC_REQUIRE(g->epilogue != CC_EPI_SPLITK || (g->Cf && g->splits >= 1), "cc_gemm_mx8_wide: split-K needs Cf");
  CC_REQUIRE(g->epilogue != CC_EPI_STORE || g->ldc >= g->N, "cc_gemm_mx8_wide: ldc >= N");
  CC_REQUIRE(!g->relu && !g->colsum && !g->H, "cc_gemm_mx8_wide: no relu / colsum / mask");
  CC_REQUIRE((int64_t)g->M * g->lda < 0x80000000ll && (int64_t)g->N * g->ldb < 0x80000000ll,
             "cc_gemm_mx8_wide: operands below 2 GB (32-bit buffer offsets)");
  CC_REQUIRE((((uintptr_t)g->A | (uintptr_t)g->B) & 15) == 0 && (((uintptr_t)g->a_scale | (uintptr_t)g->b_scale) & 3) == 0,
             "cc_gemm_mx8_wide: operands 16-B, scales 4-B aligned");
  p.A = (const uint8_t *)g->A;
  p.B = (const uint8_t *)g->B;
  p.sa = g->a_scale;
  p.sb = g->b_scale;
  p.bias = g->bias;
  p.C = (bf16_t *)g->C;
  p.Cf = g->Cf;
  p.M = g->M;
  p.N = g->N;
  p.K = g->K;
  p.lda = g->lda;
  p.ldb = g->ldb;
  p.ldc = g->ldc;
  p.epi = g->epilogue;
  p.y_bits = g->y_bits;
  p.Ct = (bf16_t *)g->Ct;
  p.ldct = g->ldct;
  p.loss_partials = g->loss_partials;
  p.loss_out = g->epilogue == CC_EPI_BCE ? g->loss_out : nullptr;
  p.ticket = g->ticket;
  p.loss_scale = g->loss_scale;
  p.scale = g->scale;
  p.zq = p.zqs = p.ztq = p.ztqs = nullptr;
  p.colsum = nullptr;
  p.ldzq = p.ldztq = 0;
  p.splits = g->epilogue == CC_EPI_SPLITK ? g->splits : 1;
  p.kchunk = (int)cdiv(cdiv(g->K, p.splits), 128) * 128;   // (128: the partition of the 128-k tiles)
  p.tiles_m = (int)cdiv(g->M, QM);
  p.ntiles = p.tiles_m * (int)cdiv(g->N, QN);
  p.a_bytes = (uint32_t)((int64_t)g->M * g->lda);
  p.b_bytes = (uint32_t)((int64_t)g->N * g->ldb);
  p.sa_bytes = (uint32_t)((int64_t)g->M * (g->lda / 32));
  p.sb_bytes = (uint32_t)((int64_t)g->N * (g->ldb / 32));
  return CC_OK;
}

bool q_attr() {
  static const bool ok = hipFuncSetAttribute((const void *)mx8_wide_kernel<false>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, QLDS) == hipSuccess &&
                         hipFuncSetAttribute((const void *)mx8_wide_kernel<true>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, QLDS_MAX) == hipSuccess &&
                         hipFuncSetAttribute((const void *)mx8_wide_pair_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, QLDS) == hipSuccess &&
                         hipFuncSetAttribute((const void *)mx8_bce_pair_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, QLDS_MAX) == hipSuccess;
  return ok;
}

__global__ __launch_bounds__(256) void colsum_zero_kernel(float *__restrict__ c, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) c[i] = 0.f;
}

}  // namespace

extern "C" int cc_gemm_mx8_wide(const cc_gemm_args *g0, const cc_gemm_args *g1, void *stream) {
  QP p0, p1;
  if (int rc = q_params(g0, p0)) return rc;
  if (g1)
    if (int rc = q_params(g1, p1)) return rc;
  CC_REQUIRE(!g1 || (p0.epi != CC_EPI_BCE && p1.epi != CC_EPI_BCE), "cc_gemm_mx8_wide: no BCE in a pair");
  CC_REQUIRE(p0.epi != CC_EPI_BCE || (int64_t)p0.M * p0.ldc * 2 < 0x100000000ll, "cc_gemm_mx8_wide: dZ below 4 GB");
  CC_REQUIRE(q_attr(), "cc_gemm_mx8_wide: dynamic LDS attribute");
  hipStream_t s = as_stream(stream);
  if (!g1) {
    if (p0.epi == CC_EPI_BCE)
      hipLaunchKernelGGL(mx8_wide_kernel<true>, dim3((unsigned)p0.ntiles), dim3(QNT), QLDS_MAX, s, p0);
    else
      hipLaunchKernelGGL(mx8_wide_kernel<false>, dim3((unsigned)(p0.ntiles * p0.splits)), dim3(QNT), QLDS, s, p0);
    CC_LAUNCH_CHECK("mx8_wide_kernel");
    return CC_OK;
  }
  hipLaunchKernelGGL(mx8_wide_pair_kernel, dim3((unsigned)(p0.ntiles * p0.splits + p1.ntiles * p1.splits)),
                     dim3(QNT), QLDS, s, p0, p1);
  CC_LAUNCH_CHECK("mx8_wide_pair_kernel");
  return CC_OK;
}

// The decoder output layer's BCE product with the MX-FP8 images of dZ made in the epilogue
// (config 5): logits -> BCE -> dz, then zq / zqs (K = N, for the dX product), ztq / ztqs (K = M,
// for the dW product) and the bias gradient colsum = column sums of the bf16 dZ, bit-exact with
// cc_quant_mx8 of the bf16 dZ / dZ^T (the column sums to fp32 rounding).  g->C / g->Ct optional.
extern "C" int cc_gemm_mx8_bce_q(const cc_gemm_args *g, uint8_t *zq, int32_t ldzq, uint8_t *zqs, uint8_t *ztq,
                                 int32_t ldztq, uint8_t *ztqs, float *colsum, void *stream) {
  return cc_gemm_mx8_bce_q2(g, zq, ldzq, zqs, ztq, ldztq, ztqs, colsum, nullptr, stream);
}

extern "C" int cc_gemm_mx8_bce_q2(const cc_gemm_args *g, uint8_t *zq, int32_t ldzq, uint8_t *zqs, uint8_t *ztq,
                                  int32_t ldztq, uint8_t *ztqs, float *colsum, const cc_gemm_args *gx,
                                  void *stream) {
  CC_REQUIRE(g && g->epilogue == CC_EPI_BCE, "cc_gemm_mx8_bce_q: BCE epilogue");
  CC_REQUIRE(zq && zqs && ztq && ztqs && colsum, "cc_gemm_mx8_bce_q: null output");
  CC_REQUIRE(ldzq % 128 == 0 && ldzq >= g->N && ldzq <= (int)cdiv(g->N, QN) * QN && ldztq % 32 == 0 && ldztq >= g->M,
             "cc_gemm_mx8_bce_q: ldzq % 128, N <= ldzq <= 256-tile cover of N; ldztq % 32, >= M");
  CC_REQUIRE(g->M % 32 == 0 && g->M <= 2 * QM, "cc_gemm_mx8_bce_q: M % 32 == 0, M <= 512 (two row tiles)");
  CC_REQUIRE((((uintptr_t)zq | (uintptr_t)ztq) & 7) == 0, "cc_gemm_mx8_bce_q: code images 8-B aligned");
  cc_gemm_args g2 = *g;
  QP p;
  const bool has_c = g->C != nullptr;
  if (!has_c) g2.C = (void *)zq;  // placeholder for the argument checks; not written
  if (int rc = q_params(&g2, p)) return rc;
  if (!has_c) p.C = nullptr;
  p.zq = zq;
  p.zqs = zqs;
  p.ztq = ztq;
  p.ztqs = ztqs;
  p.colsum = colsum;
  p.ldzq = ldzq;
  p.ldztq = ldztq;
  CC_REQUIRE(q_attr(), "cc_gemm_mx8_bce_q: dynamic LDS attribute");
  hipStream_t s = as_stream(stream);
  QP p2;
  if (gx) {
    if (int rc = q_params(gx, p2)) return rc;
    CC_REQUIRE(p2.epi != CC_EPI_BCE, "cc_gemm_mx8_bce_q2: the second problem STORE or SPLITK");
  }
  if (p.tiles_m > 1) {   // (a kernel, not hipMemsetAsync: the same node kind eagerly and in a captured graph)
    hipLaunchKernelGGL(colsum_zero_kernel, dim3((unsigned)cdiv(g->N, 256)), dim3(256), 0, s, colsum, g->N);
    CC_LAUNCH_CHECK("colsum_zero_kernel");
  }
  if (gx) {
    hipLaunchKernelGGL(mx8_bce_pair_kernel, dim3((unsigned)(p.ntiles + p2.ntiles * p2.splits)), dim3(QNT), QLDS_MAX,
                       s, p, p2);
    CC_LAUNCH_CHECK("mx8_bce_pair_kernel");
    return CC_OK;
  }
  hipLaunchKernelGGL(mx8_wide_kernel<true>, dim3((unsigned)p.ntiles), dim3(QNT), QLDS_MAX, s, p);
  CC_LAUNCH_CHECK("mx8_wide_kernel<bce>");
  return CC_OK;
}

