// D1 output layer, fused: logits -> sigmoid/BCE -> dZ -> dWo, dbo in ONE pass over a 96-column
// slice of |V| (model.py:64 Dense(V) + :94 sigmoid; train.py:85 binary_crossentropy; the
// MatMul/BiasAdd gradients of the reconstruct layer inside fit).
//
// A block owns output columns [n0, n0 + 96) for ALL B batch rows, so the output-layer weight
// gradient of those columns is complete inside the block:
//   phase 1  z[B][96] = D3[B][d] Wo^T[96][d]^T + bo   (Wo^T slice resident in LDS, D3 fragments
//            loaded global -> registers), BCE on the accumulators, dZ written row-major for the dX
//            product (cc_gemm split-K), and kept in LDS as dZ^T [96][B] (bf16, the rounded values
//            the dX product also sees) — the dZ^T HBM round trip of the unfused path is gone;
//   phase 2  dWo[d][96] = D3^T[d][B] dZ[B][96]          (D3^T fragments from global through a
//            4-deep register ring, dZ^T from LDS), dbo = colsum.
// bf16 MFMA v_mfma_f32_32x32x16_bf16 (fp32 accumulation), 8 waves; the loss is published per block
// and the last block (agent-scope ticket) reduces the partials in block order — deterministic.
#include "common.hpp"

// dev-only timing hook (tools/micro/dec_probe.hip defines it); compiled out of the library
#ifndef DEC_PROBE
#define DEC_PROBE(k)
#endif

namespace {

// V columns per block: d <= 256: 96 (ceil(22000 / 96) = 230 blocks <= 256 CUs, one round);
// d = 512 (the reference width, model.py:62-64): 64, so the Wo^T slice and dZ^T fit the LDS
template <int D> constexpr int nb_of() { return D <= 256 ? 96 : 64; }
constexpr int NB_MIN = 64;
constexpr int BK = 64;      // k per phase-2 ring chunk
constexpr int NTH = 512;    // 8 waves
constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
// cache policy of the dZ and dWo stores: default (measured, r03 / r05: non-temporal dZ slows the
// next dX kernel, which reads dZ from L2, 16 -> 19 us; non-temporal dWo neutral)
constexpr int DEC_CPOL = 0;
// The two waves of a SIMD run the VALU-bound BCE epilogue together; issue arbitration favours the
// older one, so waves 4-7 finish ~3.6 us later and the barrier after phase 1 waits for them (probe:
// tools/micro/dec_probe2.hip).  In pass ps the half (w >> 2) == (ps & 1) runs at s_setprio 1, so
// the half that lagged in pass 0 leads in pass 1 (DMA kernels).  (Round 5 measured the alternatives —
// three other priority modes, the target words staged before the A prefetch or with the Wo slice,
// the epilogue in scalar instead of packed fp32 ops, the odd dz row by a shift instead of d16_hi —
// all within +-0.3 us; they live on branch archive/r05-ab-knobs.)

typedef __attribute__((ext_vector_type(4))) uint32_t v4u;  // staging registers (stay in VGPRs)
typedef __attribute__((address_space(3))) void lds_void;
typedef short v4s __attribute__((ext_vector_type(4)));

struct DecOutP {
  const bf16_t *D3;        // [B][d]
  const bf16_t *D3t;       // [d][ldt]
  const bf16_t *D3p;       // optional packed A images (cc_tower_args.act6p / act6tp; ldt rows)
  const bf16_t *D3tp;
  const bf16_t *WoT;       // [V][d], or null: the slice is transposed from Wo in LDS
  const bf16_t *Wo;        // [d][V] (the bf16 shadow of the reconstruct kernel)
  const float *bo;         // [V]
  const uint32_t *y_bits;  // [B][ceil(V/32)]
  const uint32_t *y_img;   // or null: y_bits as cc_tower_args.y_img ([ceil(V/32)][B], register row order)
  bf16_t *dZ;              // [B][V]
  float *gW;               // [d][V]
  float *gb;               // [V]
  double *loss_partials;   // [gridDim.x]
  double *loss_out;        // [1] or null
  uint32_t *ticket;
  double loss_scale;
  float scale;
  float log2e;             // log2(e), passed in (an SGPR operand of the packed multiply)
  int V, ldt;
  int ldz;                 // dZ row pitch (elements, >= V; a multiple of 64 keeps every dZ row 128-B aligned)
};

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// element offset of (row, k) in a k-contiguous LDS image with `chunks` 16-B chunks per row,
// chunk index XOR-swizzled by the row's low 4 bits (conflict-free fragment reads)
__device__ __forceinline__ int sw_off(int row, int k, int chunks) {
  return row * chunks * 8 + ((((k >> 3) ^ (row & 15)) << 3) | (k & 7));
}

__device__ __forceinline__ bf16x8_t frag(const bf16_t *S, int off) {
  return *reinterpret_cast<const bf16x8_t *>(S + off);
}

__device__ __forceinline__ uint16_t bf16_bits(float f) {  // RNE (v_cvt_pk_bf16_f32), finite inputs
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
// x ^ (m & 0x80000000): the sign of x flipped by bit 31 of m — ONE v_bitop3_b32 (LUT 0x78 = a ^ (b & c))
__device__ __forceinline__ uint32_t xor_sign(uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(x, m, 0x80000000u, 0x78);
}
// two floats -> one packed bf16 pair (lo = a, hi = b), RNE: ONE v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t bf16_pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}

// DMA = true (d <= 256, V % 8 == 0: every Wo row segment 16-B aligned): the Wo slice is copied
// global -> LDS by buffer_load_dwordx4 ... lds as raw rows Wk[d][NB] (192 B: the tr-read banks of
// 4 consecutive k rows are disjoint, no swizzle) — no VGPR round trip and no transposing LDS
// writes; phase 1 takes its B fragments from Wk with ds_read_b64_tr_b16 (column n, 4 consecutive
// k per read).  (Measured and dropped with it: the target words by 4-B LDS-DMA as [row][NJ] — the
// epilogue's strided reads cost more than the staging saved — and phase 2 with the operands swapped
// for 16-B dWo stores: 32 rows x 32 B per store instruction ran slower than 2 x 128-B rows of
// 4-B stores; tools/micro/dec_probe2.hip)
template <int D, int BB, bool DMA, bool IMG = false>
__global__ __launch_bounds__(NTH) void dec_bce_dw_kernel(DecOutP p) {
  constexpr int d = D, B = BB;
  constexpr int NB = nb_of<D>(), NJ = NB / 32;    // slice columns, 32-column accumulators per wave
  constexpr int CHD = d / 8, CHB = B / 8;
  constexpr int nkk = d / 16;                     // 16-k steps of phase 1
  // SPLIT2 (d = 256, B = 512): phase 2 in two parts.  The dZ rows of waves 0-3 (K chunks 0, 1, 4, 5
  // of 64 rows) are ready while waves 4-7 — which lose the VALU arbitration of the shared SIMDs —
  // are still in their epilogue; waves 0-3 multiply them then (their d tile w and the partner's
  // w + 4, the partner's partial handed over through LDS), and after the barrier each wave adds
  // only the other half's chunks 2, 3, 6, 7 of its own tile: half the MFMAs after the barrier.
  constexpr bool SPLIT2 = d == 256 && B == 512;
  constexpr int npass = (B + 255) / 256;          // 256-row passes of phase 1
  // phase-1 A fragments: d <= 256 holds a whole pass (and the next one in flight); d = 512 walks
  // a ring of 16 through the pass's 32 k-steps
  constexpr bool RING1 = nkk > 16;
  constexpr int NAF = RING1 ? 16 : nkk;
  // LDS map (bytes): the Wo^T slice [NB][d] (DMA: Wo rows [d][NB]); dZ^T [NB][B].  The target bits
  // never enter the LDS: the epilogue uses them as lane masks straight from SGPRs (below)
  static_assert(!DMA || NB == 96, "dec_bce_dw_kernel: the DMA staging assumes 96-column slices");
  constexpr int ZT_OFF = NB * d * 2, ZT_BYTES = NB * B * 2;
  constexpr int LDS_BYTES = ZT_OFF + ZT_BYTES;
  static_assert(LDS_BYTES <= 150 * 1024, "dec_bce_dw_kernel: LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  __shared__ float red_cs[NTH / 64][NB];
  __shared__ double red_loss[NTH / 64];
  __shared__ int lastflag;
  __shared__ int cnt_wt, cnt_z;   // SPLIT2 hand-offs between the wave halves (LDS counters)
  // the slice's bias as MFMA B fragments: k = 0, 1, 2 carry the exact three-bf16 split of bo
  // (hi + mid + lo == bo in fp32), so one MFMA against a ones A fragment starts the accumulators at
  // the bias with no per-element moves (the epilogue is VALU-bound; the MFMA pipe has room)
  __shared__ __attribute__((aligned(16))) bf16_t bfr[NJ * 64 * 8];
  bf16_t *Wt = reinterpret_cast<bf16_t *>(smem);                 // [NB][d]
  bf16_t *Zt = reinterpret_cast<bf16_t *>(smem + ZT_OFF);        // [NB][B]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5;
  const int wu = __builtin_amdgcn_readfirstlane(w);   // the wave index as a scalar (uniform addresses)
  // the slice from an XCD-contiguous run (common.hpp): the target words' lines (32 words = ~10
  // slices) and the Wo lines two slices share are then fetched into one L2, not all 8
  // (tools/micro/d1_fetch_cal.hip: 11.2 + 17.0 of the launch's 32.8 MB of line fetches)
  const int sl = cc_slice_of_block(blockIdx.x, gridDim.x), n0 = sl * NB;
  const int V = p.V;
  const int VW = (V + 31) >> 5;

  DEC_PROBE(0);
  // pass 0's A fragments first: their L2 round trip overlaps the resident staging below
  bf16x8_t af[RING1 ? 1 : 2][NAF];
  // fragment (row block, kk): packed = 1 KB contiguous (whole cache lines per wave load).  Buffer
  // loads: the lane part is one VGPR offset computed once, the row block and k step ride in the
  // scalar offset (no per-load 64-bit address arithmetic on the VALU the epilogue is bound by)
  const bool pka = p.D3p != nullptr;
  const __amdgpu_buffer_rsrc_t a_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(pka ? p.D3p : p.D3), (short)0, (uint32_t)B * (uint32_t)d * 2u, 0x00020000);
  const int astr = pka ? 1024 : 32;   // bytes per 16-k step
  const uint32_t a_vo = pka ? (uint32_t)lane * 16u : (uint32_t)((lane & 31) * d + 8 * half) * 2u;
  auto a_so = [&](int pass) -> uint32_t {   // (uniform) byte offset of the pass's row block
    return pka ? (uint32_t)min(pass * 8 + wu, B / 32 - 1) * (uint32_t)(nkk * 1024)
               : (uint32_t)min(pass * 256 + wu * 32, B - 32) * (uint32_t)(d * 2);
  };
  auto a_ld = [&](uint32_t so, int kk) -> bf16x8_t {
    return __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(a_rs, a_vo, so + (uint32_t)(kk * astr), 0));
  };
  auto load_a = [&](bf16x8_t (&dst)[NAF], int pass) {
    const uint32_t so = a_so(pass);
#pragma unroll
    for (int kk = 0; kk < NAF; ++kk) dst[kk] = a_ld(so, kk);
    // keep the whole batch in flight: without this fence the scheduler sinks each load to its
    // MFMA and the pass becomes a chain of dependent L2 round trips
    __builtin_amdgcn_sched_barrier(0);
  };
  load_a(af[0], 0);
  // ---- resident operands: Wo^T slice (rows clamped at the edge: they feed masked columns only)
  // and the target bits; every load of the batch issued before the first LDS store
  if constexpr (DMA) {
    // Wo rows k, columns [n0, n0 + 96) -> Wk[k][96]: chunk q = 12 k + c (16 B) of the image is
    // lane q % 64 of DMA instruction q / 64; columns past V read the next row (masked columns
    // only) and rows past d read zeros (beyond the descriptor's range)
    constexpr int NI = d * 12 / 64 / (NTH / 64);   // DMA instructions per wave (6 at d = 256)
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)p.Wo, (short)0, (uint32_t)d * (uint32_t)V * 2u, 0x00020000);
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = w * NI + u, q = i * 64 + lane, k = q / 12, c = q % 12;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void *)(Wt + i * 512), 16,
                                               (uint32_t)((k * V + n0 + 8 * c) * 2), 0, 0, 0);
    }
  }
  // The target bits as lane masks: word (row, n0 / 32 + j) of y_bits holds exactly the bits of
  // the 32 columns of accumulator tile j, lane l <-> column n0 + 32 j + l.  Accumulator register r
  // of tile j holds row acc_row(r, lane) — rows rl and rl + 4 in the two lane halves — so ONE 64-bit
  // scalar (word(rl) | word(rl + 4) << 32) is that register's target mask, used directly as the
  // lane mask of v_cndmask / s_xor (inverse ballot): no per-element shift or bit extraction on
  // the VALU.  Scalar loads through the constant address space (uniform addresses; F wrote the
  // words in an earlier launch).
  typedef __attribute__((address_space(4))) const uint32_t cu32_t;
  cu32_t *yc = (cu32_t *)p.y_bits;
  // (tiles past the last word read the last word: their columns are past |V|, where the targets
  // change nothing that is kept)
  // With the image (cc_tower_args.y_img, written by the tower forward launch) a tile's 16 masks are
  // 128 contiguous bytes: two scalar 64-B loads from one address.  Without it: 32 scattered words.
  typedef __attribute__((address_space(4))) const uint64_t cu64_t;
  auto load_masks = [&](int pass, int j, uint64_t (&m)[16]) {
    const uint32_t gw = (uint32_t)min((n0 >> 5) + j, VW - 1), r0 = (uint32_t)(pass * 256 + wu * 32);
    if constexpr (IMG) {
      cu64_t *q = (cu64_t *)((cu32_t *)p.y_img + (gw * (uint32_t)B + r0));
#pragma unroll
      for (int r = 0; r < 16; ++r) m[r] = q[r];
      return;
    }
    const uint32_t base = r0 * (uint32_t)VW + gw;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t rl = (uint32_t)((r & 3) + 8 * (r >> 2));
      const uint32_t lo = yc[base + rl * (uint32_t)VW], hi = yc[base + (rl + 4) * (uint32_t)VW];
      m[r] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
  };
  {
    constexpr int NW = NB * CHD / NTH;
    // from Wo [d][V]: task = (4 consecutive k, 8 consecutive columns) -> 4 row loads, then 8
    // 8-byte LDS writes (the 4 k of one column are contiguous in the k-contiguous image);
    // columns past V clamp to V - 1
    constexpr int CN = NB / 8;                       // 16-B column chunks per Wo row segment
    constexpr int NT4 = (d / 4 * CN + NTH - 1) / NTH;  // tasks per thread
    const bool fromWo = p.WoT == nullptr;
    const bool vec = fromWo && (V % 8 == 0) && n0 + NB <= V;
    constexpr bool STAGE = !DMA;   // the Wo^T slice through registers (DMA: already in flight)
    v4u wv[fromWo ? 1 : NW];
    v4u w4[NT4][4];
    if (!STAGE) {
    } else if (!fromWo) {
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int c = tid + NTH * q, n = c / CHD, ch = c % CHD;
        wv[q] = *reinterpret_cast<const v4u *>(p.WoT + (int64_t)min(n0 + n, V - 1) * d + ch * 8);
      }
    } else {
#pragma unroll
      for (int q = 0; q < NT4; ++q) {
        const int tk = tid + NTH * q, kg = tk / CN, nc = tk % CN;
        if (kg >= d / 4) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bf16_t *row = p.Wo + (int64_t)(4 * kg + r) * V;
          if (vec) {
            w4[q][r] = *reinterpret_cast<const v4u *>(row + n0 + nc * 8);
          } else {  // ragged edge block: element loads
            uint32_t w2[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              w2[e] = (uint32_t)row[min(n0 + nc * 8 + 2 * e, V - 1)] |
                      ((uint32_t)row[min(n0 + nc * 8 + 2 * e + 1, V - 1)] << 16);
            w4[q][r] = v4u{w2[0], w2[1], w2[2], w2[3]};
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!STAGE) {
    } else if (!fromWo) {
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int c = tid + NTH * q, n = c / CHD, ch = c % CHD;
        *reinterpret_cast<v4u *>(Wt + sw_off(n, ch * 8, CHD)) = wv[q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < NT4; ++q) {
        const int tk = tid + NTH * q, kg = tk / CN, nc = tk % CN;
        if (kg >= d / 4) continue;
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // column nc*8 + e, rows 4kg .. 4kg+3
          const int sh = 16 * (e & 1);
          const uint32_t x0 = (w4[q][0][e >> 1] >> sh) & 0xFFFFu, x1 = (w4[q][1][e >> 1] >> sh) & 0xFFFFu;
          const uint32_t x2 = (w4[q][2][e >> 1] >> sh) & 0xFFFFu, x3 = (w4[q][3][e >> 1] >> sh) & 0xFFFFu;
          *reinterpret_cast<uint2 *>(Wt + sw_off(nc * 8 + e, 4 * kg, CHD)) = make_uint2(x0 | (x1 << 16), x2 | (x3 << 16));
        }
      }
    }
  }

  // ---- phase 1: logits, BCE, dZ (global + LDS dZ^T), bias-gradient partial, loss.  Wave w owns
  // rows pass*256 + 32w .. +32 and all NB columns; its A fragments (16 B per lane per 16-k step)
  // come straight from global/L2 into registers, the next pass's in flight during this one.
  float rsum = 0.f, lsum = 0.f, cs[NJ];
  bool valid[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int gc = n0 + j * 32 + (lane & 31);
    valid[j] = gc < V;
    cs[j] = 0.f;
  }
  if (tid < NJ * 64) {
    const int gc = n0 + (tid >> 6) * 32 + (tid & 31);
    const float b = ((tid & 32) == 0 && gc < V) ? p.bo[gc] : 0.f;
    const __bf16 hi = (__bf16)b;
    const float r1 = b - (float)hi;
    const __bf16 mid = (__bf16)r1;
    const __bf16 lo = (__bf16)(r1 - (float)mid);
    const __bf16 z0 = (__bf16)0.f;
    *reinterpret_cast<bf16x8_t *>(bfr + tid * 8) = bf16x8_t{hi, mid, lo, z0, z0, z0, z0, z0};
  }
  bf16x8_t ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)(half == 0 && e < 3 ? 1.f : 0.f);
  if (tid == 0) {
    cnt_wt = 0;
    cnt_z = 0;
  }
  // LDS-only barrier: __syncthreads would also wait for pass 0's A fragments (vmcnt counts loads).
  // DMA: the wave's own DMAs (issued after pass 0's A fragments) must have landed first
  if constexpr (DMA) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  DEC_PROBE(1);
  const float scale = p.scale;
  const f32x2_t l2e = {p.log2e, p.log2e};   // (a kernel argument: the packed multiply takes it from SGPRs)
  // dZ and gW through buffer descriptors: a 32-bit byte offset per store instead of a 64-bit
  // address (dZ = B x V x 2 B < 2 GB and gW = d x V x 4 B < 4 GB: checked on the host)
  const __amdgpu_buffer_rsrc_t dz_rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)p.dZ, (short)0, (uint32_t)B * (uint32_t)p.ldz * 2u, 0x00020000);
  const int LZ = p.ldz;
  // dz of rows (r2, r2 + 1) as one packed bf16 pair -> two 2-B stores (row offsets as the scalar
  // soffset); the odd row by buffer_store_short_d16_hi straight from the pair (inline asm: the
  // compiler counts no vmcnt for it — a later counted wait can only over-wait, never under-wait,
  // since this store is younger than every load it counts).  Lanes of columns past |V| carry an
  // offset beyond the descriptor's range: the hardware drops their stores (no branch)
#ifdef DEC_DIAG_NODZ   // diagnostic builds only (tools/micro/dec_probe2.hip): no dz stores
#define DEC_STORE_PAIR(PK, R2) do { (void)(PK); } while (0)
#else
#define DEC_STORE_PAIR(PK, R2)                                                                           \
  do {                                                                                                    \
    const uint32_t so0 = 2u * (uint32_t)((((R2) & 3) + 8 * ((R2) >> 2)) * LZ);                           \
    const uint32_t so1 = 2u * (uint32_t)(((((R2) + 1) & 3) + 8 * (((R2) + 1) >> 2)) * LZ);                \
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(PK), dz_rs, zv, so0, DEC_CPOL);                     \
    asm volatile("buffer_store_short_d16_hi %0, %1, %2, %3 offen" ::"v"(PK), "v"(zv), "s"(dz_rs), "s"(so1)   \
                 : "memory");                                                                             \
  } while (0)
#endif
#pragma unroll
  for (int ps = 0; ps < npass; ++ps) {
    if (!RING1 && ps + 1 < npass) load_a(af[(ps + 1) & 1], ps + 1);
    if (ps * 256 + w * 32 >= B) continue;          // wave-uniform: rows beyond B
    f32x16_t acc[NJ];  // starts at the bias (exactly): z = bo + sum_k D3 Wo accumulates in the MFMA
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, *reinterpret_cast<const bf16x8_t *>(bfr + (j * 64 + lane) * 8),
                                                       f32x16_t{}, 0, 0, 0);
    const uint32_t aso = a_so(ps);
#pragma unroll
    for (int kk = 0; kk < nkk; ++kk) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        bf16x8_t b;
        if constexpr (DMA) {   // column n = 32 j + (lane & 31), k = 16 kk + 8 half + 0..7: two transposed reads
          const bf16_t *tb = Wt + (kk * 16 + 8 * half + ((lane >> 2) & 3)) * NB + j * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)tb);
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)(tb + 4 * NB));
          b = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        } else {
          b = frag(Wt, sw_off(j * 32 + (lane & 31), kk * 16 + 8 * half, CHD));
        }
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[RING1 ? 0 : ps & 1][kk % NAF], b, acc[j], 0, 0, 0);
      }
      if (RING1 && kk + NAF < nkk) af[0][kk % NAF] = a_ld(aso, kk + NAF);
    }
    if (RING1 && ps + 1 < npass) load_a(af[0], ps + 1);   // the next pass's head under this epilogue
    DEC_PROBE(2 + 2 * ps);
    if constexpr (SPLIT2) {
      if (ps == npass - 1) {   // this wave reads the Wo slice no more (its fragment reads returned)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(&cnt_wt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    if constexpr (DMA && npass > 1) {   // the half (w >> 2) == (ps & 1) leads pass ps (wave-uniform)
      if ((wu >> 2) == (ps & 1))
        __builtin_amdgcn_s_setprio(1);
      else
        __builtin_amdgcn_s_setprio(0);
    }
    const int rb = ps * 256 + w * 32;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uint64_t mk[16];   // this tile's target masks (the other wave of the SIMD covers their latency)
      load_masks(ps, j, mk);
      const int col = j * 32 + (lane & 31);
      uint32_t tt[8];  // dz of rows (r, r+1) as one packed bf16 pair (one v_cvt_pk_bf16_f32)
      // sigmoid_cross_entropy_with_logits (TF 2.5 Keras BCE on a sigmoid output):
      //   loss = max(z, 0) - z y + log1p(exp(-|z|)),  dz = (sigmoid(z) - y) / (B V)
      // in the target-signed logit s = (1 - 2y) z:
      //   loss = max(s, 0) + log1p(exp(-|s|)),  dz = (1 - 2y) sigmoid(s) / (B V)
      // (sigmoid(z) - 1 = -sigmoid(-z)), so sigmoid(s) never cancels against y.  The sign of s is
      // a lane mask: [z < 0] (one compare into SGPRs) xor the target mask (a scalar op); then
      // max(s, 0) = s < 0 ? 0 : |z|, sigmoid(s) = s < 0 ? a / (1 + a) : 1 / (1 + a) and dz's sign
      // are one v_cndmask each (|z|, -x as source modifiers).  a = exp(-|z|) = exp2(-|z log2 e|)
      // (the product packed for two rows, abs / neg folded into v_exp); log1p and 1/(1+a) from it.
      // The 16 factors 1 + a in (1, 2] of a lane's column are multiplied (<= 2^16) and one log2
      // per column taken: the log is a quarter-rate instruction; summed log2 scaled by ln 2 at the
      // end.  Columns past |V| (the last slice) compute on clamped operands: their stores are
      // dropped (zv) and their loss is masked per tile; their dZ^T columns feed only dWo columns
      // that are never stored
      // store offsets: the lane part in a VGPR, the row part (r) as the scalar soffset
      const uint32_t zv = valid[j] ? 2u * (uint32_t)((rb + 4 * half) * LZ + n0 + col) : 0x80000000u;
      f32x2_t lprod = {1.f, 1.f}, rs2 = {0.f, 0.f}, cs2 = {0.f, 0.f};  // even / odd rows: packed math
#pragma unroll
      for (int r2 = 0; r2 < 16; r2 += 2) {
        const f32x2_t z2 = {acc[j][r2], acc[j][r2 + 1]};
        const f32x2_t zl = z2 * l2e;
        f32x2_t a2, rl2, sel2, dzp;
        bool yb[2], sn[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          yb[e] = __builtin_amdgcn_inverse_ballot_w64(mk[r2 + e]);
          sn[e] = (z2[e] < 0.f) != yb[e];   // s < 0
          a2[e] = __builtin_amdgcn_exp2f(-fabsf(zl[e]));
          rl2[e] = sn[e] ? 0.f : fabsf(z2[e]);
        }
        const f32x2_t opa2 = 1.f + a2;
        f32x2_t rp2;
#pragma unroll
        for (int e = 0; e < 2; ++e) rp2[e] = __builtin_amdgcn_rcpf(opa2[e]);
        lprod *= opa2;
        rs2 += rl2;
        const f32x2_t arp2 = a2 * rp2;
#pragma unroll
        for (int e = 0; e < 2; ++e) sel2[e] = sn[e] ? arp2[e] : rp2[e];   // sigmoid(s)
        const f32x2_t mag2 = sel2 * scale;
#pragma unroll
        for (int e = 0; e < 2; ++e) dzp[e] = yb[e] ? -mag2[e] : mag2[e];
        cs2 += dzp;   // the bias gradient sums the fp32 dz (the reference's arithmetic)
        const uint32_t pk = bf16_pack2(dzp[0], dzp[1]);
        tt[r2 >> 1] = pk;
        DEC_STORE_PAIR(pk, r2);
      }
      lsum += valid[j] ? __builtin_amdgcn_logf(lprod[0] * lprod[1]) : 0.f;
      rsum += valid[j] ? rs2[0] + rs2[1] : 0.f;
      cs[j] += cs2[0] + cs2[1];
      // dZ^T image: registers 4g..4g+3 = 4 consecutive rows -> one 8-byte LDS store
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<uint2 *>(Zt + sw_off(col, rb + 8 * g + 4 * half, CHB)) = make_uint2(tt[2 * g], tt[2 * g + 1]);
    }
    DEC_PROBE(3 + 2 * ps);
  }
  if constexpr (DMA && npass > 1) __builtin_amdgcn_s_setprio(0);
  if constexpr (SPLIT2) {   // waves 0-3: this wave's dZ^T rows are in LDS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (w < 4 && lane == 0) __hip_atomic_fetch_add(&cnt_z, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }

  // bias gradient: column sums of dz in a fixed order (lane halves, then waves)
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float c2 = cs[j] + __shfl_xor(cs[j], 32);
    if (half == 0) red_cs[w][j * 32 + (lane & 31)] = c2;
  }
  float lossf = rsum + lsum * LN2;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) lossf += __shfl_xor(lossf, off);
  if (lane == 0) red_loss[w] = (double)lossf;
  const bool pk = p.D3tp != nullptr;
  if constexpr (SPLIT2) {
    // A fragment (chunk kc, step kk) of d tile t: 1 KB contiguous from the packed D3^T image, or
    // row-strided from D3^T (buffer loads: lane part in one VGPR, tile / chunk / step as the
    // scalar offset — both layouts put tile t at t * ldt * 64 bytes)
    const __amdgpu_buffer_rsrc_t t_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(pk ? p.D3tp : p.D3t), (short)0, (uint32_t)d * (uint32_t)p.ldt * 2u, 0x00020000);
    const uint32_t t_vo = pk ? (uint32_t)lane * 16u : (uint32_t)((lane & 31) * p.ldt + 8 * half) * 2u;
    auto af_t = [&](int t, int kc, int kk) -> bf16x8_t {
      const uint32_t so = (uint32_t)t * (uint32_t)p.ldt * 64u + (pk ? (uint32_t)(kc * 4 + kk) * 1024u : (uint32_t)(kc * BK + kk * 16) * 2u);
      return __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(t_rs, t_vo, so, 0));
    };
    const bool fast = wu < 4;   // (wave-uniform)
    f32x16_t acc2[NJ];
    // the partner's partial: 16 x 64 fp32 per 32-column tile, [j][group g][lane][4]
    float *part = reinterpret_cast<float *>(smem) + (w & 3) * (NJ * 16 * 64);
    static_assert(4 * NJ * 16 * 64 * 4 <= ZT_OFF, "dec_bce_dw_kernel: partials fit the Wo slice's LDS");
    if (fast) {
      f32x16_t accx[NJ];
      constexpr int KF[4] = {0, 1, 4, 5};
      bf16x8_t fa[2][4], fx[2][4];   // two chunks in flight
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          fa[q][kk] = af_t(wu, KF[q], kk);
          fx[q][kk] = af_t(wu + 4, KF[q], kk);
        }
      while (__hip_atomic_load(&cnt_z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4) __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int kc = KF[c], q = c & 1;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const bf16x8_t b = frag(Zt, sw_off(j * 32 + (lane & 31), kc * BK + kk * 16 + 8 * half, CHB));
            const bool first = c == 0 && kk == 0;   // (static: the accumulators start at zero)
            acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q][kk], b, first ? f32x16_t{} : acc2[j], 0, 0, 0);
            accx[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fx[q][kk], b, first ? f32x16_t{} : accx[j], 0, 0, 0);
          }
        if (c + 2 < 4) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            fa[q][kk] = af_t(wu, KF[c + 2], kk);
            fx[q][kk] = af_t(wu + 4, KF[c + 2], kk);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // the Wo slice's LDS is free once every wave is past its phase-1 MFMAs
      while (__hip_atomic_load(&cnt_wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < NTH / 64) __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4_t *>(part + ((j * 4 + g) * 64 + lane) * 4) =
              f32x4_t{accx[j][4 * g], accx[j][4 * g + 1], accx[j][4 * g + 2], accx[j][4 * g + 3]};
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[j][r] = 0.f;
    }
    // this wave's own tile, the slow half's chunks: fragments in flight across the barrier
    constexpr int KS[4] = {2, 3, 6, 7};
    bf16x8_t fs[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) fs[c][kk] = af_t(wu, KS[c], kk);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // dZ^T rows, partials, red_cs, red_loss
    DEC_PROBE(6);
    if (tid < NB && n0 + tid < V) {
      float g = 0.f;
      for (int i = 0; i < NTH / 64; ++i) g += red_cs[i][tid];
      p.gb[n0 + tid] = g;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const bf16x8_t b = frag(Zt, sw_off(j * 32 + (lane & 31), KS[c] * BK + kk * 16 + 8 * half, CHB));
          acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fs[c][kk], b, acc2[j], 0, 0, 0);
        }
    if (!fast) {   // + the fast partner's chunks 0, 1, 4, 5 of this tile
      const float *pp = reinterpret_cast<const float *>(smem) + (w & 3) * (NJ * 16 * 64);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4_t x = *reinterpret_cast<const f32x4_t *>(pp + ((j * 4 + g) * 64 + lane) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc2[j][4 * g + e] += x[e];
        }
    }
    DEC_PROBE(7);
    const int dr0 = w * 32;
    const __amdgpu_buffer_rsrc_t gw_rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)p.gW, (short)0, (uint32_t)d * (uint32_t)V * 4u, 0x00020000);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int gc2 = n0 + j * 32 + (lane & 31);
      if (gc2 < V) {
        uint32_t g0 = (uint32_t)((dr0 + 4 * half) * V + gc2);
        asm volatile("" : "+v"(g0));
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc2[j][r]), gw_rs,
                                                4u * (g0 + (uint32_t)(((r & 3) + 8 * (r >> 2)) * V)), 0, DEC_CPOL);
      }
    }
  } else {
  // phase 2's first A fragments in flight before the barrier.  The barrier waits for LDS only:
  // __syncthreads' release fence would also drain every wave's dZ stores (vmcnt(0), ~4 us), and
  // nothing below reads them.
  constexpr int P2D = 4;
  constexpr int nk2 = B / BK;
  constexpr int ND2 = (d + 255) / 256;   // 32-row d tiles per wave: w (and w + 8 at d = 512)
  // A fragment (kc, kk) of d tile dt: row-strided from D3^T, or 1 KB contiguous from the packed
  // image (buffer loads: lane part in one VGPR, tile / chunk / step as the scalar offset — both
  // layouts put tile t at t * ldt * 64 bytes)
  const __amdgpu_buffer_rsrc_t t_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(pk ? p.D3tp : p.D3t), (short)0, (uint32_t)d * (uint32_t)p.ldt * 2u, 0x00020000);
  const uint32_t t_vo = pk ? (uint32_t)lane * 16u : (uint32_t)((lane & 31) * p.ldt + 8 * half) * 2u;
  uint32_t t_so = (uint32_t)min(wu, d / 32 - 1) * (uint32_t)p.ldt * 64u;
  auto afrag = [&](int kc, int kk) -> bf16x8_t {
    const uint32_t so = t_so + (pk ? (uint32_t)(kc * 4 + kk) * 1024u : (uint32_t)(kc * BK + kk * 16) * 2u);
    return __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(t_rs, t_vo, so, 0));
  };
  bf16x8_t ring[P2D][4];
  auto fill_ring = [&]() {
#pragma unroll
    for (int q = 0; q < P2D; ++q)
      if (q < nk2)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) ring[q][kk] = afrag(q, kk);
  };
  fill_ring();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // dZ^T image, red_cs, red_loss
  DEC_PROBE(6);
  if (tid < NB && n0 + tid < V) {
    float g = 0.f;
    for (int i = 0; i < NTH / 64; ++i) g += red_cs[i][tid];
    p.gb[n0 + tid] = g;
  }

  // ---- phase 2: dWo[d][NB] = D3^T[d][B] . dZ[B][NB].  Wave w owns rows 32w .. +32 of d (and
  // 32(w + 8) .. at d = 512; waves beyond d idle) and all NB columns; A fragments from global
  // through a ring P2D chunks of 64 k
  // deep, B fragments from the dZ^T image.
#pragma unroll 1
  for (int dt = 0; dt < ND2 && (w + 8 * dt) * 32 < d; ++dt) {
    if (dt > 0) {
      t_so = (uint32_t)min(wu + 8 * dt, d / 32 - 1) * (uint32_t)p.ldt * 64u;
      fill_ring();
    }
    const int dr0 = (w + 8 * dt) * 32;   // this tile's first row of dWo
    f32x16_t acc2[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[j][r] = 0.f;
#pragma unroll
    for (int kc = 0; kc < nk2; ++kc) {
      const int q = kc % P2D;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const bf16x8_t b = frag(Zt, sw_off(j * 32 + (lane & 31), kc * BK + kk * 16 + 8 * half, CHB));
          acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ring[q][kk], b, acc2[j], 0, 0, 0);
        }
      }
      if (kc + P2D < nk2) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) ring[q][kk] = afrag(kc + P2D, kk);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    DEC_PROBE(7);
    const __amdgpu_buffer_rsrc_t gw_rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)p.gW, (short)0, (uint32_t)d * (uint32_t)V * 4u, 0x00020000);
    {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int gc2 = n0 + j * 32 + (lane & 31);
        if (gc2 < V) {
          uint32_t g0 = (uint32_t)((dr0 + 4 * half) * V + gc2);
          asm volatile("" : "+v"(g0));
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc2[j][r]), gw_rs,
                                                  4u * (g0 + (uint32_t)(((r & 3) + 8 * (r >> 2)) * V)), 0, DEC_CPOL);
        }
      }
    }
  }

  }

  // loss: the block partial, published after phase 2's stores (the ticket's vmcnt(0) drains them)
  if (tid == 0) {
    double sum = 0.0;
    for (int i = 0; i < NTH / 64; ++i) sum += red_loss[i];
    lastflag = 0;
    if (!p.loss_out) {
      p.loss_partials[sl] = sum;
    } else {
      __hip_atomic_store(&p.loss_partials[sl], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t tk = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lastflag = tk == gridDim.x - 1;
    }
  }
  DEC_PROBE(8);
  // ---- the last block reduces the loss partials in slice order
  if (p.loss_out) {
    __syncthreads();
    if (lastflag) {
      double s2d = 0.0;
      for (int i = tid; i < (int)gridDim.x; i += NTH)
        s2d += __hip_atomic_load(&p.loss_partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s2d += __shfl_xor(s2d, off);
      if (lane == 0) red_loss[w] = s2d;
      __syncthreads();
      if (tid == 0) {
        double tot = 0.0;
        for (int i = 0; i < NTH / 64; ++i) tot += red_loss[i];
        p.loss_out[0] = tot * p.loss_scale;
        __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

}  // namespace

static int dec_bce_dw_launch(const void *D3, const void *D3t, int32_t ldt, const void *D3p, const void *D3tp,
                             const void *WoT, const void *Wo, const float *bo, int32_t B, int32_t d, int32_t V,
                             const uint32_t *y_bits, const uint32_t *y_img, void *dZ, int32_t ldz, float *gW,
                             float *gb, double *loss_partials, double *loss_out, double loss_scale,
                             uint32_t *ticket, void *stream) {
  // (dZ below 2 GB: the stores of columns past |V| carry the byte offset 2^31, beyond the range)
  CC_REQUIRE(ldz >= V && (int64_t)B * ldz * 2 <= 0x7FFFFFFFll, "cc_dec_bce_dw: ldz >= V, dZ below 2 GB");
  CC_REQUIRE(D3 && D3t && (WoT || Wo) && bo && y_bits && dZ && gW && gb && loss_partials,
             "cc_dec_bce_dw: null pointer");
  CC_REQUIRE(B == 128 || B == 256 || B == 512, "cc_dec_bce_dw: B must be 128, 256 or 512");
  CC_REQUIRE(d == 128 || d == 256 || d == 512, "cc_dec_bce_dw: d must be 128, 256 or 512");
  CC_REQUIRE(V > 0 && ldt >= B && ldt % 8 == 0, "cc_dec_bce_dw: V > 0, ldt >= B, ldt % 8 == 0");
  CC_REQUIRE((int64_t)d * V * 4 <= 0xFFFFFFFFll, "cc_dec_bce_dw: dWo below 4 GB (32-bit buffer offsets)");
  CC_REQUIRE(!loss_out || ticket, "cc_dec_bce_dw: loss_out needs a ticket word");
  CC_REQUIRE((((uintptr_t)D3 | (uintptr_t)D3t | (uintptr_t)WoT | (uintptr_t)Wo) & 15) == 0,
             "cc_dec_bce_dw: operands 16-B aligned");
  DecOutP p;
  p.D3 = (const bf16_t *)D3;
  p.D3t = (const bf16_t *)D3t;
  p.D3p = (const bf16_t *)D3p;
  p.D3tp = (const bf16_t *)D3tp;
  CC_REQUIRE(!D3tp || ldt % 16 == 0, "cc_dec_bce_dw: packed D3^T needs ldt % 16 == 0");
  CC_REQUIRE((((uintptr_t)D3p | (uintptr_t)D3tp) & 15) == 0, "cc_dec_bce_dw: packed images 16-B aligned");
  p.WoT = (const bf16_t *)WoT;
  p.Wo = (const bf16_t *)Wo;
  p.bo = bo;
  p.y_bits = y_bits;
  CC_REQUIRE((((uintptr_t)y_img) & 127) == 0, "cc_dec_bce_dw: y_img 128-B aligned");
  p.y_img = y_img;
  p.dZ = (bf16_t *)dZ;
  p.gW = gW;
  p.gb = gb;
  p.loss_partials = loss_partials;
  p.loss_out = loss_out;
  p.ticket = ticket;
  p.loss_scale = loss_scale;
  p.scale = 1.0f / ((float)B * (float)V);
  p.log2e = LOG2E;
  p.V = V;
  p.ldt = ldt;
  p.ldz = ldz;
  const dim3 grid((unsigned)cdiv(V, d <= 256 ? nb_of<256>() : nb_of<512>())), block(NTH);
  hipStream_t s = as_stream(stream);
  // the DMA staging: Wo read in place with every row segment 16-B aligned (V % 8 == 0), the
  // 96-column slices of d <= 256
  const bool dma = Wo != nullptr && WoT == nullptr && V % 8 == 0 && d <= 256 && (((uintptr_t)y_bits) & 3) == 0 &&
                   (int64_t)d * V * 2 <= 0xFFFFFFFFll && (int64_t)B * ((V + 31) / 32) * 4 <= 0xFFFFFFFFll;
#define DO_LAUNCH(DD, BBB)                                                                    \
  if (d == DD && B == BBB) {                                                                  \
    if (dma && DD <= 256 && p.y_img)                                                          \
      hipLaunchKernelGGL((dec_bce_dw_kernel<DD, BBB, DD <= 256, true>), grid, block, 0, s, p); \
    else if (dma && DD <= 256)                                                                \
      hipLaunchKernelGGL((dec_bce_dw_kernel<DD, BBB, DD <= 256>), grid, block, 0, s, p);      \
    else                                                                                      \
      hipLaunchKernelGGL((dec_bce_dw_kernel<DD, BBB, false>), grid, block, 0, s, p);          \
  }
  DO_LAUNCH(256, 512) DO_LAUNCH(256, 256) DO_LAUNCH(256, 128)
  DO_LAUNCH(128, 512) DO_LAUNCH(128, 256) DO_LAUNCH(128, 128)
  DO_LAUNCH(512, 512) DO_LAUNCH(512, 256) DO_LAUNCH(512, 128)
#undef DO_LAUNCH
  CC_LAUNCH_CHECK("dec_bce_dw_kernel");
  return CC_OK;
}

extern "C" int cc_dec_bce_dw_ld(const void *D3, const void *D3t, int32_t ldt, const void *D3p,
                                const void *D3tp, const void *WoT, const void *Wo,
                                const float *bo, int32_t B, int32_t d, int32_t V, const uint32_t *y_bits,
                                void *dZ, int32_t ldz, float *gW, float *gb, double *loss_partials,
                                double *loss_out, double loss_scale, uint32_t *ticket, void *stream) {
  return dec_bce_dw_launch(D3, D3t, ldt, D3p, D3tp, WoT, Wo, bo, B, d, V, y_bits, nullptr, dZ, ldz, gW, gb,
                           loss_partials, loss_out, loss_scale, ticket, stream);
}

extern "C" int cc_dec_bce_dw_img(const void *D3, const void *D3t, int32_t ldt, const void *D3p,
                                 const void *D3tp, const void *WoT, const void *Wo,
                                 const float *bo, int32_t B, int32_t d, int32_t V, const uint32_t *y_bits,
                                 const uint32_t *y_img, void *dZ, int32_t ldz, float *gW, float *gb,
                                 double *loss_partials, double *loss_out, double loss_scale, uint32_t *ticket,
                                 void *stream) {
  CC_REQUIRE(y_img, "cc_dec_bce_dw_img: null y_img");
  return dec_bce_dw_launch(D3, D3t, ldt, D3p, D3tp, WoT, Wo, bo, B, d, V, y_bits, y_img, dZ, ldz, gW, gb,
                           loss_partials, loss_out, loss_scale, ticket, stream);
}

extern "C" int cc_dec_bce_dw(const void *D3, const void *D3t, int32_t ldt, const void *D3p,
                             const void *D3tp, const void *WoT, const void *Wo,
                             const float *bo, int32_t B, int32_t d, int32_t V, const uint32_t *y_bits,
                             void *dZ, float *gW, float *gb, double *loss_partials, double *loss_out,
                             double loss_scale, uint32_t *ticket, void *stream) {
  return cc_dec_bce_dw_ld(D3, D3t, ldt, D3p, D3tp, WoT, Wo, bo, B, d, V, y_bits, dZ, V, gW, gb, loss_partials,
                          loss_out, loss_scale, ticket, stream);
}

// an upper bound over every d (the narrowest slice)
extern "C" int32_t cc_dec_bce_dw_blocks(int32_t V) { return (int32_t)cdiv(V, NB_MIN); }
