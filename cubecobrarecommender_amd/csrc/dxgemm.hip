// Decoder dX product, split-K with an LDS-DMA pipeline: P[s][M][N] = A[M][k in split s] . B[N][..]^T,
// A = dZ [M][lda] bf16 (the output-layer gradient, K = |V|), B = Wo [N][ldb] bf16 (the reconstruct
// kernel as stored, [d][V]: k-contiguous) — the Dense(V) input gradient of model.py:64 inside fit.
//
// The shape (M = 512 rows, N = d = 256, K = 22,000) gives 8 output tiles of 128 x 128, so the chip
// is filled by splitting K (32 splits: 256 workgroups, ~11 K-tiles each).  With so few K-tiles per
// workgroup the register-staged NT kernel (gemm.hip) never reaches a steady state: its 2-3 tiles
// in flight do not cover one L2/MALL round trip.  Here every K-tile (A 128 x 64 + B 128 x 64 bf16,
// 32 KB) is copied global -> LDS by buffer_load_dwordx4 ... lds (no VGPR staging), four LDS stages
// deep (three tiles in flight while the fourth is multiplied), counted vmcnt waits and raw
// s_barrier (a __syncthreads would drain the DMA queue).  The LDS images are lane-linear per wave
// instruction (8 rows x 128 B); the 16-B chunk XOR swizzle (chunk ^ (row >> 1 & 7)) is applied on
// the global source address.  (row >> 1, not row: a ds_read_b128 is serviced in four lane groups of
// 16 — lanes {0-3, 12-15, 20-27}, ... — whose rows r and r + 8 / r + 24 share a 16-B bank slot under
// chunk ^ (row & 7), a 2-way conflict on every fragment read; under (row >> 1 & 7) the 16 rows of
// each group land on 16 distinct slots: SQ_LDS_BANK_CONFLICT 30 M -> 0 per dx_wide launch (r05x,
// r05y); the kernel's time did not move with them — its fragment reads were not its bound.)  k >= kend chunks point past the buffer's range: the DMA writes zeros.
// (tile, split) pairs are dealt split-major over the 8 XCDs so a split's A and B panels are
// fetched into one XCD's L2 once.  The split partials are summed by cc_splitk_reduce.
#include <cstdlib>

#include "common.hpp"

// build knob (A/B builds: CCREC_EXTRA_FLAGS=-DCCREC_DX_WIDE_MIN=..., a tagged library; no run-time switch)
#ifndef CCREC_DX_WIDE_MIN
#define CCREC_DX_WIDE_MIN 4096
#endif

namespace {

constexpr int XBM = 128, XBN = 128, XBK = 64, XST = 4, XNT = 256;
constexpr int XTILE_BYTES = (XBM + XBN) * XBK * 2;  // one stage: A then B, 32 KB
constexpr int XLDS = XST * XTILE_BYTES;             // 128 KB

__device__ __forceinline__ int xcd_remap(int b, int nb) {  // bijective blocks -> XCD-contiguous ids
  const int q = nb / 8, r = nb % 8, x = b % 8, slot = b / 8;
  return x < r ? x * (q + 1) + slot : r * (q + 1) + (x - r) * q + slot;
}

typedef __attribute__((address_space(3))) void lds_void;

struct DxP {
  const bf16_t *A, *B;
  float *P;
  int M, N, K, lda, ldb, splits, kchunk, tiles_m;
  uint32_t a_bytes, b_bytes;
};

// issue the DMA of K-tile (k0) into stage buffer st: wave w moves A rows [32w, 32w+32) and B rows
// [32w, 32w+32) as 4 + 4 instructions of 8 rows x 128 B
__device__ __forceinline__ void dma_tile(const DxP &p, const __amdgpu_buffer_rsrc_t &ra,
                                         const __amdgpu_buffer_rsrc_t &rb, char *smem, int st, int bm,
                                         int bn, int k0, int kend) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rl = lane >> 3, slot = lane & 7;
  char *sa = smem + st * XTILE_BYTES, *sb = sa + XBM * XBK * 2;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = w * 4 + u;       // instruction index: rows 8i .. 8i + 7
    const int row = 8 * i + rl;
    const int c = slot ^ ((row >> 1) & 7);
    const int k = k0 + 8 * c;
    const uint32_t oa = k < kend ? (uint32_t)(((bm + row) * p.lda + k) * 2) : 0x80000000u;
    const uint32_t ob = k < kend ? (uint32_t)(((bn + row) * p.ldb + k) * 2) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void *)(sa + i * 1024), 16, oa, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void *)(sb + i * 1024), 16, ob, 0, 0, 0);
  }
}

template <int N_OUT>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N_OUT == 16)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N_OUT == 8)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ bf16x8_t frag(const char *s, int row, int c) {  // 16 B: row, k-chunk c
  return *reinterpret_cast<const bf16x8_t *>(s + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
}

__global__ __launch_bounds__(XNT) void dx_splitk_kernel(DxP p) {
  __shared__ __attribute__((aligned(1024))) char smem[XLDS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int ntiles = p.tiles_m * (p.N / XBN);
  const int q = xcd_remap(blockIdx.x, ntiles * p.splits);
  const int split = q / ntiles, tile = q % ntiles;
  const int bm = (tile % p.tiles_m) * XBM, bn = (tile / p.tiles_m) * XBN;
  const int kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
  const int nk = kbeg < kend ? (kend - kbeg + XBK - 1) / XBK : 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)p.A, (short)0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)p.B, (short)0, p.b_bytes, 0x00020000);
  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // prologue: XST - 1 tiles in flight
#pragma unroll
  for (int s = 0; s < XST - 1; ++s)
    if (s < nk) dma_tile(p, ra, rb, smem, s, bm, bn, kbeg + s * XBK, kend);
  const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31);
  for (int t = 0; t < nk; ++t) {
    // tile t landed in every wave (own DMAs counted, then the barrier); 8 DMA instructions per
    // wave per tile, min(2, nk - 1 - t) tiles issued after t may stay in flight
    const int after = min(XST - 2, nk - 1 - t);
    if (after >= 2)
      wait_vm<16>();
    else if (after == 1)
      wait_vm<8>();
    else
      wait_vm<0>();
    __builtin_amdgcn_s_barrier();   // raw barrier: a __syncthreads fence would drain the DMA queue
    asm volatile("" ::: "memory");  // no LDS read or DMA issue moves across it
    // every wave finished reading buffer (t - 1) % XST in iteration t - 1: refill it with t + 3
    if (t + XST - 1 < nk) dma_tile(p, ra, rb, smem, (t + XST - 1) % XST, bm, bn, kbeg + (t + XST - 1) * XBK, kend);
    const char *sa = smem + (t % XST) * XTILE_BYTES, *sb = sa + XBM * XBK * 2;
#pragma unroll
    for (int kk = 0; kk < XBK / 16; ++kk) {
      const int c = 2 * kk + half;
      const bf16x8_t a0 = frag(sa, ar, c), a1 = frag(sa, ar + 32, c);
      const bf16x8_t b0 = frag(sb, br, c), b1 = frag(sb, br + 32, c);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  // partial tile -> P[split][M][N] (lanes 0..31 of a half: 32 consecutive columns of one row)
  float *out = p.P + (int64_t)split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = bn + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = bm + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        out[(int64_t)row * p.N + col] = acc[i][j][r];
      }
    }
}

// ---- the tall shape (the full-mode regulariser: M = |V| identity rows, N = d = 256): 128 x 256
// tiles, so each dZ panel (the 968 MB operand at |V| = 22,000) is read from HBM once instead of
// once per 128-column tile; 8 waves as 2 (M) x 4 (N) of 64 x 64, 3 LDS stages of A 128 x 64 +
// B 256 x 64 (48 KB each).  Splits are dealt split-major over the XCDs as above, so a split's Wo
// panel (256 x K/splits bf16) stays in one XCD's L2.
constexpr int WBM = 128, WBN = 256, WST = 3, WNT = 512;
// dev diagnostics (tools/micro/dx_diag.hip; 0 in the library): 1 no Wo copies / fragment loads, 2 no dZ
// copies, 4 no MFMA (dx_wide_kernel and dx_wide3_kernel)
#ifndef DXW_DIAG
#define DXW_DIAG 0
#endif
constexpr int WTILE_BYTES = (WBM + WBN) * XBK * 2;  // 48 KB
constexpr int WLDS = WST * WTILE_BYTES;              // 144 KB

// stage st <- K-tile k0: A rows [0, 128) (2 instructions per wave) and B rows [0, 256) (4 per wave),
// each instruction 8 rows x 128 B
__device__ __forceinline__ void dma_tile_w(const DxP &p, const __amdgpu_buffer_rsrc_t &ra,
                                           const __amdgpu_buffer_rsrc_t &rb, char *smem, int st, int bm,
                                           int bn, int k0, int kend) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rl = lane >> 3, slot = lane & 7;
  char *sa = smem + st * WTILE_BYTES, *sb = sa + WBM * XBK * 2;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if constexpr (DXW_DIAG & 2) break;
    const int i = w * 2 + u;  // A rows 8i .. 8i + 7
    const int row = 8 * i + rl;
    const int k = k0 + 8 * (slot ^ ((row >> 1) & 7));
    const uint32_t oa = k < kend ? (uint32_t)(((bm + row) * p.lda + k) * 2) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void *)(sa + i * 1024), 16, oa, 0, 0, 2);  // dZ is read once: non-temporal
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if constexpr (DXW_DIAG & 1) break;
    const int i = w * 4 + u;  // B rows 8i .. 8i + 7
    const int row = 8 * i + rl;
    const int k = k0 + 8 * (slot ^ ((row >> 1) & 7));
    const uint32_t ob = k < kend ? (uint32_t)(((bn + row) * p.ldb + k) * 2) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void *)(sb + i * 1024), 16, ob, 0, 0, 0);
  }
}

__global__ __launch_bounds__(WNT) void dx_wide_kernel(DxP p) {
  extern __shared__ __attribute__((aligned(1024))) char wsmem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5;
  const int wm = w >> 2, wn = w & 3;
  const int ntiles = p.tiles_m * (p.N / WBN);
  const int q = xcd_remap(blockIdx.x, ntiles * p.splits);
  const int split = q / ntiles, tile = q % ntiles;
  const int bm = (tile % p.tiles_m) * WBM, bn = (tile / p.tiles_m) * WBN;
  const int kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
  const int nk = kbeg < kend ? (kend - kbeg + XBK - 1) / XBK : 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)p.A, (short)0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)p.B, (short)0, p.b_bytes, 0x00020000);
  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
  for (int s = 0; s < WST - 1; ++s)
    if (s < nk) dma_tile_w(p, ra, rb, wsmem, s, bm, bn, kbeg + s * XBK, kend);
  const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31);
  for (int t = 0; t < nk; ++t) {
    // tile t landed (own DMAs counted, then the barrier); 6 DMA instructions per wave per tile,
    // min(1, nk - 1 - t) tiles issued after t may stay in flight
    if (t + 1 < nk)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + WST - 1 < nk) dma_tile_w(p, ra, rb, wsmem, (t + WST - 1) % WST, bm, bn, kbeg + (t + WST - 1) * XBK, kend);
    const char *sa = wsmem + (t % WST) * WTILE_BYTES, *sb = sa + WBM * XBK * 2;
#pragma unroll
    for (int kk = 0; kk < XBK / 16; ++kk) {
      if constexpr (DXW_DIAG & 4) {
        const int c = 2 * kk + half;
        acc[0][0][0] += __builtin_bit_cast(float, __builtin_shufflevector(frag(sa, ar, c), frag(sb, br, c), 0, 9));
        continue;
      }
      const int c = 2 * kk + half;
      const bf16x8_t a0 = frag(sa, ar, c), a1 = frag(sa, ar + 32, c);
      const bf16x8_t b0 = frag(sb, br, c), b1 = frag(sb, br + 32, c);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  float *out = p.P + (int64_t)split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = bn + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = bm + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        out[(int64_t)row * p.N + col] = acc[i][j][r];
      }
    }
}

// ---- the tall shape with Wo from its packed fragment image (cc_pack_frag_b): only the dZ tile goes
// through LDS (LDS-DMA, 16 KB per K-tile, three stages); each wave owns 32 columns of N and all 128
// rows and loads its Wo fragments — 1 KB per wave instruction, one fragment (32 columns x 16 k) per
// load — one K-tile ahead into registers: each Wo element once per block, fully coalesced, no LDS
// round trip (dx_wide_kernel: copies 361 of its 388 us; the same loads from the row-major Wo, 16 B
// from each of 32 rows per instruction, were slower: 440).  Per K-tile and wave: B(t + 1) loads,
// then DMA(t + 2), so the counted wait for B(t) does not wait on the newest copies; copies and
// loads past the end use the range sentinel (zeros, no traffic) so every iteration issues the same
// count.  The MFMA chain per output is the other paths' (bit-identical partials).
#ifndef DX3_LEAD
#define DX3_LEAD 2   // build knob: dZ K-tiles copied ahead of the one multiplied (stages = lead + 1)
#endif
#ifndef DX3_CPOL
#define DX3_CPOL 0   // build knob: the dZ copies' cache policy (default; nt measured 343 vs 304 us)
#endif
constexpr int W3L = DX3_LEAD, W3ST = W3L + 1, W3NT = 512;
static_assert(W3L >= 2 && W3L <= 5, "dx_wide3: the startup waits below are written for leads 2..5");

template <int N>
__device__ __forceinline__ void w2_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
constexpr int W3TILE = WBM * XBK * 2;   // 16 KB: the dZ tile only

__global__ __launch_bounds__(W3NT) void dx_wide3_kernel(DxP p) {
  extern __shared__ __attribute__((aligned(1024))) char w3mem[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), half = lane >> 5;
  const int ntiles = p.tiles_m * (p.N / WBN);
  const int q = xcd_remap(blockIdx.x, ntiles * p.splits);
  const int split = q / ntiles, tile = q % ntiles;
  const int bm = (tile % p.tiles_m) * WBM, bn = (tile / p.tiles_m) * WBN;
  const int kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
  const int nk = kbeg < kend ? (kend - kbeg + XBK - 1) / XBK : 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)p.A, (short)0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)p.B, (short)0, p.b_bytes, 0x00020000);
  const int rl = lane >> 3, slot = lane & 7;
  auto dma = [&](int t) {   // dZ K-tile t -> stage t % W3ST: 2 instructions of 8 rows x 128 B per wave
    if constexpr (DXW_DIAG & 2) return;
    char *sa = w3mem + (t % W3ST) * W3TILE;
    const int k0 = kbeg + t * XBK;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = w * 2 + u, row = 8 * i + rl;
      const int k = k0 + 8 * (slot ^ ((row >> 1) & 7));
      const uint32_t oa = k < kend ? (uint32_t)(((bm + row) * p.lda + k) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void *)(sa + i * 1024), 16, oa, 0, 0, DX3_CPOL);   // dZ: default policy (knob)
    }
  };
  // fragment (band, k step) of the packed image: 1 KB at (band * nks + k step) KB, lane L's 16 B at 16 L
  const int nks = (p.K + 15) / 16;
  const uint32_t bbase = (uint32_t)((bn / 32 + w) * nks) * 1024u + 16u * (uint32_t)lane;
  auto bload = [&](bf16x8_t (&dst)[XBK / 16], int t) {   // Wo fragments of K-tile t
    if constexpr (DXW_DIAG & 1) return;
    const int k0 = kbeg + t * XBK;
#pragma unroll
    for (int ks = 0; ks < XBK / 16; ++ks) {
      const int k = k0 + 16 * ks;
      const uint32_t ob = k < kend ? bbase + (uint32_t)(k / 16) * 1024u : 0x80000000u;
      dst[ks] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(rb, ob, 0, 0));
    }
  };
  f32x16_t acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  bf16x8_t bf[2][XBK / 16];
  // prologue: DMA(0 .. L - 1), then B(0) (sched barriers: the waits count on the issue order).
  // Per K-tile t: wait for DMA(t), barrier, B(t + 1) (4 loads), DMA(t + L) (2).  The accesses
  // younger than DMA(t) at that wait: 6 (L - 1) in the steady state; at t < L - 2 (the prologue's
  // later copies, B(0) and t tiles) 2 L + 2 + 4 t, fewer — those waits use their own counts.
#pragma unroll
  for (int j = 0; j < W3L; ++j) dma(j);
  __builtin_amdgcn_sched_barrier(0);
  bload(bf[0], 0);
  __builtin_amdgcn_sched_barrier(0);
  const int ar = lane & 31;
  auto body = [&](bf16x8_t (&cur)[XBK / 16], bf16x8_t (&nxt)[XBK / 16], int t) {
    if (W3L >= 3 && t == 0)
      w2_wait<(2 * W3L + 2) % 64>();
    else if (W3L >= 4 && t == 1)
      w2_wait<(2 * W3L + 6) % 64>();
    else if (W3L >= 5 && t == 2)
      w2_wait<(2 * W3L + 10) % 64>();
    else
      w2_wait<6 * (W3L - 1)>();   // own DMA(t) landed
    __builtin_amdgcn_s_barrier();   // every wave's DMA(t) landed; stage (t - 1) % W3ST read by all
    asm volatile("" ::: "memory");
    bload(nxt, t + 1);
    __builtin_amdgcn_sched_barrier(0);
    dma(t + W3L);
    __builtin_amdgcn_sched_barrier(0);
    const char *sa = w3mem + (t % W3ST) * W3TILE;
#pragma unroll
    for (int ks = 0; ks < XBK / 16; ++ks) {
      const int c = 2 * ks + half;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (DXW_DIAG & 4)
          acc[i][0] += __builtin_bit_cast(float, __builtin_shufflevector(frag(sa, ar + 32 * i, c), cur[ks], 0, 9));
        else
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(sa, ar + 32 * i, c), cur[ks], acc[i], 0, 0, 0);
      }
    }
  };
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    body(bf[0], bf[1], t);
    body(bf[1], bf[0], t + 1);
  }
  if (t < nk) body(bf[0], bf[1], t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing copies land before the LDS is released
  float *out = p.P + (int64_t)split * p.M * p.N;
  const int n = bn + 32 * w + (lane & 31);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = bm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      out[(int64_t)row * p.N + n] = acc[i][r];
    }
  }
}

// B [N][K] bf16 (row pitch ldb) -> MFMA B-fragment image [N / 32][ceil(K / 16)][64 lanes][8]: lane L
// of fragment (band, k step) holds B[32 band + (L & 31)][16 k step + 8 (L >> 5) ..][8]; k >= K zero
__global__ __launch_bounds__(256) void pack_frag_b_kernel(const bf16_t *__restrict__ B, int N, int K, int ldb,
                                                          uint4 *__restrict__ dst) {
  const int nks = (K + 15) / 16;
  const int64_t total = (int64_t)(N / 32) * nks * 64;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int lane = (int)(i & 63);
    const int64_t f = i >> 6;
    const int band = (int)(f / nks), ks = (int)(f % nks);
    const int n = 32 * band + (lane & 31), k = 16 * ks + 8 * (lane >> 5);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (k < K) v = *reinterpret_cast<const uint4 *>(B + (int64_t)n * ldb + k);   // (K % 8 == 0)
    dst[i] = v;
  }
}

}  // namespace

extern "C" size_t cc_pack_frag_b_size(int32_t N, int32_t K) { return (size_t)(N / 32) * ((K + 15) / 16) * 1024; }

extern "C" int cc_pack_frag_b(const void *B, int32_t N, int32_t K, int32_t ldb, void *dst, void *stream) {
  CC_REQUIRE(B && dst && N > 0 && N % 32 == 0 && K > 0 && K % 8 == 0 && ldb % 8 == 0 && ldb >= K,
             "cc_pack_frag_b: N % 32, K % 8, ldb % 8, ldb >= K");
  CC_REQUIRE((((uintptr_t)B | (uintptr_t)dst) & 15) == 0, "cc_pack_frag_b: 16-B aligned");
  hipLaunchKernelGGL(pack_frag_b_kernel, dim3(2048), dim3(256), 0, as_stream(stream), (const bf16_t *)B, N, K, ldb,
                     (uint4 *)dst);
  CC_LAUNCH_CHECK("pack_frag_b_kernel");
  return CC_OK;
}

extern "C" int cc_gemm_dx_splitk_pk(const void *A, int32_t lda, const void *Bp, int32_t M, int32_t N, int32_t K,
                                    int32_t splits, float *partials, void *stream) {
  CC_REQUIRE(A && Bp && partials, "cc_gemm_dx_splitk_pk: null pointer");
  CC_REQUIRE(M > 0 && N > 0 && M % WBM == 0 && N % WBN == 0, "cc_gemm_dx_splitk_pk: M % 128, N % 256");
  CC_REQUIRE(K > 0 && K % 8 == 0 && lda % 8 == 0 && lda >= K, "cc_gemm_dx_splitk_pk: K, lda multiples of 8, lda >= K");
  CC_REQUIRE(splits >= 1 && splits <= 1024, "cc_gemm_dx_splitk_pk: splits 1..1024");
  CC_REQUIRE((int64_t)M * lda * 2 < 0x80000000ll && (int64_t)cc_pack_frag_b_size(N, K) < 0x80000000ll,
             "cc_gemm_dx_splitk_pk: operands below 2 GB (32-bit buffer offsets)");
  CC_REQUIRE((((uintptr_t)A | (uintptr_t)Bp) & 15) == 0, "cc_gemm_dx_splitk_pk: operands 16-B aligned");
  DxP p;
  p.A = (const bf16_t *)A;
  p.B = (const bf16_t *)Bp;
  p.P = partials;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = 0;
  p.splits = splits;
  p.kchunk = (int)cdiv(cdiv(K, splits), XBK) * XBK;
  p.tiles_m = M / WBM;
  p.a_bytes = (uint32_t)((int64_t)M * lda * 2);
  p.b_bytes = (uint32_t)cc_pack_frag_b_size(N, K);
  static bool attr3 = [] {
    return hipFuncSetAttribute((const void *)dx_wide3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               W3ST * W3TILE) == hipSuccess;
  }();
  CC_REQUIRE(attr3, "cc_gemm_dx_splitk_pk: dynamic LDS attribute");
  const int nb = (M / WBM) * (N / WBN) * splits;
  hipLaunchKernelGGL(dx_wide3_kernel, dim3((unsigned)nb), dim3(W3NT), W3ST * W3TILE, as_stream(stream), p);
  CC_LAUNCH_CHECK("dx_wide3_kernel");
  return CC_OK;
}

extern "C" int cc_gemm_dx_splitk(const void *A, int32_t lda, const void *B, int32_t ldb, int32_t M, int32_t N,
                                 int32_t K, int32_t splits, float *partials, void *stream) {
  CC_REQUIRE(A && B && partials, "cc_gemm_dx_splitk: null pointer");
  CC_REQUIRE(M > 0 && N > 0 && M % XBM == 0 && N % XBN == 0, "cc_gemm_dx_splitk: M, N multiples of 128");
  CC_REQUIRE(K > 0 && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K,
             "cc_gemm_dx_splitk: K, lda, ldb multiples of 8, lda/ldb >= K");
  CC_REQUIRE(splits >= 1 && splits <= 1024, "cc_gemm_dx_splitk: splits 1..1024");
  CC_REQUIRE((int64_t)M * lda * 2 < 0x80000000ll && (int64_t)N * ldb * 2 < 0x80000000ll,
             "cc_gemm_dx_splitk: operands must stay below 2 GB (32-bit buffer offsets)");
  CC_REQUIRE((((uintptr_t)A | (uintptr_t)B) & 15) == 0, "cc_gemm_dx_splitk: operands 16-B aligned");
  DxP p;
  p.A = (const bf16_t *)A;
  p.B = (const bf16_t *)B;
  p.P = partials;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.splits = splits;
  p.kchunk = (int)cdiv(cdiv(K, splits), XBK) * XBK;
  p.tiles_m = M / XBM;
  p.a_bytes = (uint32_t)((int64_t)M * lda * 2);
  p.b_bytes = (uint32_t)((int64_t)N * ldb * 2);
  constexpr int wide_min = CCREC_DX_WIDE_MIN;  // build knob: smallest M for the 128 x 256 tiles (0: never)
  if (wide_min > 0 && M >= wide_min && N % WBN == 0) {  // tall M (full-mode regulariser)
    static bool attr = [] {
      return hipFuncSetAttribute((const void *)dx_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, WLDS) ==
             hipSuccess;
    }();
    CC_REQUIRE(attr, "cc_gemm_dx_splitk: dynamic LDS attribute");
    const int nb = (M / WBM) * (N / WBN) * splits;
    hipLaunchKernelGGL(dx_wide_kernel, dim3((unsigned)nb), dim3(WNT), WLDS, as_stream(stream), p);
    CC_LAUNCH_CHECK("dx_wide_kernel");
    return CC_OK;
  }
  const int nb = (M / XBM) * (N / XBN) * splits;
  hipLaunchKernelGGL(dx_splitk_kernel, dim3((unsigned)nb), dim3(XNT), 0, as_stream(stream), p);
  CC_LAUNCH_CHECK("dx_splitk_kernel");
  return CC_OK;
}
