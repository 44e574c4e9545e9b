// D2 output layer, fused: logits -> softmax -> KL against M~ rows -> dZ -> dWo, dbo, with no fp32
// logits in HBM (model.py:64 Dense(V) + :98 softmax of the decoder_for_reg branch; train.py:85
// kullback_leibler_divergence under TF 2.5's clip semantics).  The regulariser
// counterpart of decout.hip's D1 kernel; the softmax's row normaliser needs every column, so the
// logits are produced twice:
//
//   stats  (slice, 256-row group) blocks: z = D3 Wo + bo on MFMA over a 96-column slice, per-row
//          max and sum exp(z - max) of the slice -> partials [rows][slices]
//   merge  one wave per row: m = max_i m_i, s = sum_i s_i exp(m_i - m) -> {m, ln s, S, C}, where
//          S = sum_j t and C = sum_j t ln t over t = clip(M~[row], 1e-7, 1) (cc_kl_tsum, once per M~)
//   main   slice blocks over every row tile: z again, p = exp(z - m)/s, t = clip(M~ row, 1e-7, 1),
//          KL -= t ln clip(p, 1e-7, 1) (+ C once per row: KL = sum t (ln t - ln clip(p))), dz =
//          scale (p S - [p >= 1e-7] t) written row-major for the dX product and kept as dZ^T in
//          LDS -> dWo[d][96] = D3^T dZ, dbo = colsum.  Many row tiles (full mode): dWo instead by
//          kl_dwo_kernel from the stored dZ (after the fix)
//   fix    TF's gradient passes through clip only where p >= 1e-7, so the exact S is
//          S - delta, delta = sum_{p < 1e-7} t.  The main kernel writes each (row, slice)'s delta
//          partial (zero unless a wave saw such an element) and raises a flag; the fix kernel
//          (dz -= scale p delta with the matching dWo / dbo corrections) runs only then —
//          otherwise it exits at once.
//
// Padding rows (reg_idx < 0, owner-computes capacity / full-mode round-up) contribute nothing.
// bf16 MFMA v_mfma_f32_32x32x16_bf16 with fp32 accumulation; A operands from the packed D3 images
// the tower forward writes (cc_tower_args.act6p / act6tp), Wo read in place ([d][V], the slice
// transposed into LDS).  Deterministic: every sum has a fixed order.
#include <cstdlib>

#include "common.hpp"

// diagnostic builds only (tools/micro/kl_probe_full.hip): the register path without its dZ stores /
// its M~ loads (wrong results; what they cost)
#ifndef KL_DIAG_NOSTORE
#define KL_DIAG_NOSTORE 0
#endif
#ifndef KL_DIAG_NOMT
#define KL_DIAG_NOMT 0
#endif

// dev-only timing hook (tools/micro/kl_probe.hip defines it); compiled out of the library
#ifndef KL_PROBE
#define KL_PROBE(k)
#endif

namespace {

// V columns per block: d <= 256: 96 (230 slices at |V| = 22,000); d = 512 (the reference width,
// model.py:62-64): 64, so the Wo slice and the dZ^T tile fit the LDS together
template <int D> constexpr int kl_nb() { return D <= 256 ? 96 : 64; }
constexpr int NB_MIN = 64;
constexpr int NTH = 512;     // 8 waves
constexpr int TR = 512;      // rows per tile of the main kernel (2 passes of 8 x 32)
constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
constexpr float PMIN = 1e-7f;
// Cache policy of the streamed operands of the main pass (M~ rows read once, dZ written once).
// Full mode (many row tiles per slice): non-temporal for both, so they do not evict the block's
// dWo slice between its per-tile read-modify-writes — 1,620 -> 1,500 us per block
// (tools/micro/kl_probe_full.hip; either alone gains ~1 %).  One tile (the sampled regulariser):
// default — the non-temporal pair slowed its epilogues (p1 4.9 -> 6.8 us).
constexpr int KL_CPOL_NT = 2;  // the SLC/NT bit of the buffer instructions' cache-policy operand
#ifndef KL_ZST_CPOL
#define KL_ZST_CPOL -1   // build knob: the 16-B dZ row stores' policy (-1: the pass's CPOL; 0 measured
                         // 2,378 vs 2,199-2,206 us/step, r05zo: the non-temporal stores carry the gain)
#endif
#ifndef KL_SEP_CPOL
#define KL_SEP_CPOL KL_CPOL_NT   // build knob: the main pass's policy with dWo in its own kernel
#endif
constexpr float LN_PMIN = -16.11809565095832f;  // ln(1e-7)


typedef __attribute__((ext_vector_type(4))) uint32_t v4u;
typedef __attribute__((address_space(3))) void lds_void;
typedef short v4s __attribute__((ext_vector_type(4)));

struct KlP {
  int d, V, rows, ldt, row0, nsl;
  const bf16_t *D3p, *D3tp, *Wo;
  const float *bo, *Mt, *tsum;
  const int32_t *reg_idx;
  float scale;
  bf16_t *dZ;
  float *gW, *gb;
  double *loss_partials, *loss_out;
  double loss_scale;
  uint32_t *ticket;
  uint32_t mt_bytes;               // extent of Mt from its base (buffer range check)
  int mt_lo;                        // first card whose M~ row is resident
  float *part_m, *part_s, *part_d;  // [rows][nsl]
  float4 *rowstat;                  // [rows] {m + ln s, -, S, sum t ln t}
  float2 *rowst2;                   // [rows] {m + ln s, S} (the main pass's MS staging)
  uint32_t *flag;                   // [1] an element with p < 1e-7 was seen this step
  float *dw_part;                   // [d][V] kl_dwo2_kernel's first-half partial dWo
};

// Workgroup barrier over LDS only.  __syncthreads' release fence also waits for every outstanding
// global access of the wave (vmcnt(0): the dZ / dWo stores and in-flight loads) — not needed where
// only LDS is handed between the waves.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }
__device__ __forceinline__ int sw_off(int row, int k, int chunks) {
  return row * chunks * 8 + ((((k >> 3) ^ (row & 15)) << 3) | (k & 7));
}
__device__ __forceinline__ bf16x8_t frag(const bf16_t *S, int off) {
  return *reinterpret_cast<const bf16x8_t *>(S + off);
}
__device__ __forceinline__ uint16_t bf16_bits(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }


// Wo [d][V] slice [n0, n0 + NB) -> LDS k-contiguous image Wt[NB][d] (swizzled); columns past V clamp
template <int D>
__device__ __forceinline__ void load_wo_slice(const bf16_t *__restrict__ Wo, int V, int n0, bf16_t *Wt) {
  constexpr int NB = kl_nb<D>();
  constexpr int CHD = D / 8, CN = NB / 8, NT4 = (D / 4 * CN + NTH - 1) / NTH;
  const int tid = threadIdx.x;
  const bool vec = (V % 8 == 0) && n0 + NB <= V;
  v4u w4[NT4][4];
#pragma unroll
  for (int q = 0; q < NT4; ++q) {
    const int tk = tid + NTH * q, kg = tk / CN, nc = tk % CN;
    if (kg >= D / 4) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bf16_t *row = Wo + (int64_t)(4 * kg + r) * V;
      if (vec) {
        w4[q][r] = *reinterpret_cast<const v4u *>(row + n0 + nc * 8);
      } else {
        uint32_t w2[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          w2[e] = (uint32_t)row[min(n0 + nc * 8 + 2 * e, V - 1)] |
                  ((uint32_t)row[min(n0 + nc * 8 + 2 * e + 1, V - 1)] << 16);
        w4[q][r] = v4u{w2[0], w2[1], w2[2], w2[3]};
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < NT4; ++q) {
    const int tk = tid + NTH * q, kg = tk / CN, nc = tk % CN;
    if (kg >= D / 4) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int sh = 16 * (e & 1);
      const uint32_t x0 = (w4[q][0][e >> 1] >> sh) & 0xFFFFu, x1 = (w4[q][1][e >> 1] >> sh) & 0xFFFFu;
      const uint32_t x2 = (w4[q][2][e >> 1] >> sh) & 0xFFFFu, x3 = (w4[q][3][e >> 1] >> sh) & 0xFFFFu;
      *reinterpret_cast<uint2 *>(Wt + sw_off(nc * 8 + e, 4 * kg, CHD)) = make_uint2(x0 | (x1 << 16), x2 | (x3 << 16));
    }
  }
}

// z[32 rows][NB] = bo + D3[rows] Wo_slice for the wave's 32-row block rb (packed D3 image): the
// A-fragment loads (logits_load, a ring of LRING) and the MFMAs (logits_mfma) are separate so a
// caller can put other loads behind the fragments' in the memory queue
template <int D, int RG = (D / 16 < 8 ? D / 16 : 8)>
struct LFrag {
  static constexpr int nkk = D / 16, RING = RG;
  bf16x8_t af[RING];
  const bf16_t *src;
};
template <int D, int RG>
__device__ __forceinline__ void logits_load(const KlP &p, int rb, LFrag<D, RG> &f) {
  const int lane = threadIdx.x & 63;
  f.src = p.D3p + ((int64_t)rb * LFrag<D, RG>::nkk * 64 + lane) * 8;
#pragma unroll
  for (int kk = 0; kk < RG; ++kk) f.af[kk] = *reinterpret_cast<const bf16x8_t *>(f.src + kk * 512);
}
template <int D, int RG>
__device__ __forceinline__ void logits_mfma(const bf16_t *Wt, LFrag<D, RG> &f, const float (&bias)[kl_nb<D>() / 32],
                                            f32x16_t (&acc)[kl_nb<D>() / 32]) {
  constexpr int NJ = kl_nb<D>() / 32;
  constexpr int nkk = LFrag<D, RG>::nkk, RING = RG, CHD = D / 8;
  const int lane = threadIdx.x & 63, half = lane >> 5;
  // the Wo-slice fragments are the same for every row block: an opaque base per call keeps the
  // compiler from hoisting all of them (192+ VGPRs) out of the callers' row loops
  int wofs = 0;
  asm volatile("" : "+v"(wofs));
  Wt += wofs;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float b = bias[j];
    asm volatile("" : "+v"(b));  // per call: the 48-register bias broadcast is not hoisted (and spilled)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = b;
  }
#pragma unroll
  for (int kk = 0; kk < nkk; ++kk) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const bf16x8_t b = frag(Wt, sw_off(j * 32 + (lane & 31), kk * 16 + 8 * half, CHD));
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.af[kk % RING], b, acc[j], 0, 0, 0);
    }
    if (kk + RING < nkk) f.af[kk % RING] = *reinterpret_cast<const bf16x8_t *>(f.src + (kk + RING) * 512);
  }
}

// Reduce-scatter of 16 per-row values over the 32 lanes of a half-wave (lanes with the same
// lane >> 5 hold the same 16 rows of an MFMA accumulator, one column each): 8 + 4 + 2 + 1 + 1
// shuffles instead of 16 x 5.  Returns, in every lane, the reduction of row (lane >> 1) & 15.
template <bool MAX>
__device__ __forceinline__ float rs16(const float (&v)[16]) {
  const int lane = threadIdx.x & 63;
  float a[8];
  {
    const bool b = lane & 16;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float send = b ? v[i] : v[i + 8], keep = b ? v[i + 8] : v[i];
      const float got = __shfl_xor(send, 16);
      a[i] = MAX ? fmaxf(keep, got) : keep + got;
    }
  }
#pragma unroll
  for (int h = 4, m = 8; h >= 1; h >>= 1, m >>= 1) {  // xor 8, 4, 2 on 4, 2, 1 values
    const bool b = lane & m;
#pragma unroll
    for (int i = 0; i < h; ++i) {
      const float send = b ? a[i] : a[i + h], keep = b ? a[i + h] : a[i];
      const float got = __shfl_xor(send, m);
      a[i] = MAX ? fmaxf(keep, got) : keep + got;
    }
  }
  const float got = __shfl_xor(a[0], 1);
  return MAX ? fmaxf(a[0], got) : a[0] + got;
}

__device__ __forceinline__ float half_max(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// ---------------------------------------------------------------- stats
// z^T[96 cols][32 rows] per wave with the operands swapped (Wo slice = A, D3 rows = B): a lane holds
// ONE row and 16 columns per 32-column tile, so the row's max / sum over the slice are lane-local
// (+ one exchange between the lane halves).  Columns past V start at -inf (bias) and drop out of
// both.  One block per slice stages its Wo slice once; its waves walk the 32-row blocks.
template <int D>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(1, 2))) void kl_stats_kernel(KlP p) {
  constexpr int NB = kl_nb<D>(), NJ = NB / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Wt[NB * D];
  constexpr int CHD = D / 8;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5;
  const int sl = cc_slice_of_block(blockIdx.x, gridDim.x), n0 = sl * NB;
  __shared__ __attribute__((aligned(16))) float bs[NB];   // the slice's bias, -inf past V
  KL_PROBE(8);
  if (sl == 0 && threadIdx.x == 0) *p.flag = 0u;  // this step's fix flag starts clear
  if (threadIdx.x < NB) bs[threadIdx.x] = n0 + (int)threadIdx.x < p.V ? p.bo[n0 + threadIdx.x] : -INFINITY;
  load_wo_slice<D>(p.Wo, p.V, n0, Wt);
  __syncthreads();
  KL_PROBE(9);
  // wave w walks the 32-row blocks w, w + 8, ...; the next block's fragments load during this one
  // (d <= 256: two whole fragment sets; d = 512: one ring of 16 refilled during the MFMAs, the
  // next block's head loaded behind the last MFMA)
  const int nrb = p.rows / 32;
  constexpr int nkk = D / 16;
  constexpr bool RINGS = nkk > 16;
  constexpr int NAF = RINGS ? 16 : nkk;
  constexpr int W8 = NTH / 64;
  bf16x8_t af[RINGS ? 1 : 2][NAF];
  auto src_of = [&](int rb) {
    return p.D3p + ((int64_t)((p.row0 + 32 * min(rb, nrb - 1)) / 32) * nkk * 64 + lane) * 8;
  };
  auto load = [&](bf16x8_t (&dst)[NAF], int rb) {
    const bf16_t *src = src_of(rb);
#pragma unroll
    for (int kk = 0; kk < NAF; ++kk) dst[kk] = *reinterpret_cast<const bf16x8_t *>(src + kk * 512);
  };
  auto body = [&](bf16x8_t (&cur)[NAF], int rb) {
    f32x16_t acc[NJ];  // bias-initialised: registers 4g..4g+3 are columns 8g + 4 half .. +3
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b = *reinterpret_cast<const float4 *>(bs + j * 32 + 8 * g + 4 * half);
        acc[j][4 * g] = b.x;
        acc[j][4 * g + 1] = b.y;
        acc[j][4 * g + 2] = b.z;
        acc[j][4 * g + 3] = b.w;
      }
    const bf16_t *src = src_of(rb);
    int wofs = 0;   // opaque per row block: the Wo-slice fragments are not hoisted out of the loop
    asm volatile("" : "+v"(wofs));
    const bf16_t *Wtb = Wt + wofs;
#pragma unroll
    for (int kk = 0; kk < nkk; ++kk) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bf16x8_t a = frag(Wtb, sw_off(j * 32 + (lane & 31), kk * 16 + 8 * half, CHD));
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, cur[kk % NAF], acc[j], 0, 0, 0);
      }
      if (RINGS && kk + NAF < nkk) cur[kk % NAF] = *reinterpret_cast<const bf16x8_t *>(src + (kk + NAF) * 512);
    }
    if (RINGS && rb + W8 < nrb) load(cur, rb + W8);
    if (rb == w) KL_PROBE(10);
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, acc[j][r]);
    m = fmaxf(m, __shfl_xor(m, 32));
    float e = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) e += __builtin_amdgcn_exp2f((acc[j][r] - m) * LOG2E);
    e += __shfl_xor(e, 32);
    if (rb == w) KL_PROBE(11);
    if (half == 0) {
      const int row = 32 * rb + lane;
      p.part_m[(int64_t)row * p.nsl + sl] = m;
      p.part_s[(int64_t)row * p.nsl + sl] = e;
    }
  };
  load(af[0], w);
  if constexpr (RINGS) {
    for (int rb = w; rb < nrb; rb += W8) body(af[0], rb);
  } else {
    for (int rb = w; rb < nrb; rb += 2 * W8) {
      if (rb + W8 < nrb) load(af[1], rb + W8);
      __builtin_amdgcn_sched_barrier(0);
      body(af[0], rb);
      if (rb + W8 < nrb) {
        if (rb + 2 * W8 < nrb) load(af[0], rb + 2 * W8);
        __builtin_amdgcn_sched_barrier(0);
        body(af[1], rb + W8);
      }
    }
  }
}

// The same row stats with two adjacent slices per block and the rows split in two halves (the
// full-mode shape, d = 256): kl_stats_kernel's blocks each re-read all of the packed D3 (11 MB at
// |V| = 22,000, ~42 B/clk per CU of fragment loads at its MFMA rate) — the pattern kl_dwo2_kernel
// removed from the dWo product.  Here each loaded row block feeds 6 column tiles instead of 3 (half
// the D3 bytes per output), with the row block's fragments in ONE register ring (each k step's
// fragment reloaded for the wave's next row block right after its MFMAs: registers for the 6
// accumulators).  Per 96-column slice the MFMA order, the max and the sum are kl_stats_kernel's:
// the same partials bit for bit.  Grid: ceil(nsl / 2) slice pairs x 2 row halves.
#ifndef CCREC_KL_STATS2
#define CCREC_KL_STATS2 1   // build knob (A/B builds): 0 = kl_stats_kernel for every shape
#endif
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(1, 2))) void kl_stats2_kernel(KlP p) {
  constexpr int D = 256, NB = kl_nb<D>(), NJ = NB / 32, CHD = D / 8, nkk = D / 16, W8 = NTH / 64;
  __shared__ __attribute__((aligned(16))) bf16_t Wt[2][NB * D];
  __shared__ __attribute__((aligned(16))) float bs[2][NB];   // the slices' biases, -inf past V
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5;
  const int sp = blockIdx.x, rh = blockIdx.y;
  if (sp == 0 && rh == 0 && threadIdx.x == 0) *p.flag = 0u;  // this step's fix flag starts clear
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int n0 = (2 * sp + q) * NB;
    if (threadIdx.x < NB) bs[q][threadIdx.x] = n0 + (int)threadIdx.x < p.V ? p.bo[n0 + threadIdx.x] : -INFINITY;
    load_wo_slice<D>(p.Wo, p.V, min(n0, (p.nsl - 1) * NB), Wt[q]);   // (a pair past nsl: never written)
  }
  __syncthreads();
  const int nrb = p.rows / 32, rb0 = nrb * rh / 2, rb1 = nrb * (rh + 1) / 2;
  auto src_of = [&](int rb) {
    return p.D3p + ((int64_t)((p.row0 + 32 * min(rb, nrb - 1)) / 32) * nkk * 64 + lane) * 8;
  };
  bf16x8_t af[nkk];
  {
    const bf16_t *src = src_of(rb0 + w);
#pragma unroll
    for (int kk = 0; kk < nkk; ++kk) af[kk] = *reinterpret_cast<const bf16x8_t *>(src + kk * 512);
  }
  for (int rb = rb0 + w; rb < rb1; rb += W8) {
    f32x16_t acc[2][NJ];  // bias-initialised: registers 4g..4g+3 are columns 8g + 4 half .. +3
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 b = *reinterpret_cast<const float4 *>(&bs[q][j * 32 + 8 * g + 4 * half]);
          acc[q][j][4 * g] = b.x;
          acc[q][j][4 * g + 1] = b.y;
          acc[q][j][4 * g + 2] = b.z;
          acc[q][j][4 * g + 3] = b.w;
        }
    const bf16_t *nsrc = src_of(rb + W8);   // (clamped past the end: loaded, never used)
    int wofs = 0;   // opaque per row block: the Wo-slice fragments are not hoisted out of the loop
    asm volatile("" : "+v"(wofs));
#pragma unroll
    for (int kk = 0; kk < nkk; ++kk) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const bf16x8_t a = frag(Wt[q] + wofs, sw_off(j * 32 + (lane & 31), kk * 16 + 8 * half, CHD));
          acc[q][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, af[kk], acc[q][j], 0, 0, 0);
        }
      af[kk] = *reinterpret_cast<const bf16x8_t *>(nsrc + kk * 512);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) m = fmaxf(m, acc[q][j][r]);
      m = fmaxf(m, __shfl_xor(m, 32));
      float e = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) e += __builtin_amdgcn_exp2f((acc[q][j][r] - m) * LOG2E);
      e += __shfl_xor(e, 32);
      const int sl = 2 * sp + q;
      if (half == 0 && sl < p.nsl) {
        const int row = 32 * rb + lane;
        p.part_m[(int64_t)row * p.nsl + sl] = m;
        p.part_s[(int64_t)row * p.nsl + sl] = e;
      }
    }
  }
}

// ---------------------------------------------------------------- merge (one wave per row)
// The row's slice partials are loaded once (MRG per lane in registers) — one memory round trip.
constexpr int MRG = 8;  // nsl <= 512 (|V| <= 49,152): checked on the host
__global__ __launch_bounds__(256) void kl_merge_kernel(KlP p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const float *pm = p.part_m + (int64_t)row * p.nsl, *ps = p.part_s + (int64_t)row * p.nsl;
  float mv[MRG], sv[MRG];
#pragma unroll
  for (int q = 0; q < MRG; ++q) {
    const int i = lane + 64 * q;
    mv[q] = i < p.nsl ? pm[i] : -INFINITY;
    sv[q] = i < p.nsl ? ps[i] : 0.f;
  }
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < MRG; ++q) m = fmaxf(m, mv[q]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < MRG; ++q) s += sv[q] * __builtin_amdgcn_exp2f((mv[q] - m) * LOG2E);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) {
    const int card = p.reg_idx[row];
    const float2 ts = card >= 0 ? reinterpret_cast<const float2 *>(p.tsum)[card] : make_float2(0.f, 0.f);
    // (one value for both images: m + ln s contracts differently if written twice)
    const float lse = m + __logf(s);
    p.rowstat[row] = make_float4(lse, 0.f, ts.x, ts.y);   // {m + ln s, -, S, C}: ln p = z - .x
    p.rowst2[row] = make_float2(lse, ts.x);
  }
}

// ---------------------------------------------------------------- main
template <int NB>
struct MainSmem {
  bf16_t Zt[NB * TR];       // dZ^T tile [NB][TR] (swizzled); staged M~ (kl_slice's MS mode)
  float4 rs[TR];            // row stats of the tile
  int32_t card[TR];         // M~ row byte offset of the tile's rows (0x80000000: padding row)
  float red_cs[NTH / 64][NB];
  double red_loss[NTH / 64];
  int lastflag;
};

// FIX = false: the main pass.  FIX = true: the exact-clip correction (runs only when p.flag is set):
// c = -scale p delta_row replaces dz; dZ, dWo, dbo are updated in place.
// (Measured and dropped for the full-mode regulariser: keeping the block's dWo slice in the
// waves' accumulators across all row tiles instead of the per-tile gW read-modify-write — the
// 48 extra registers pushed the logits' fragment ring from 16 to 8 and spilled, and the logits
// phases then waited on L2 twice as long: 1,620 -> 2,015 us per block, tools/micro/kl_probe_full.hip.)
__device__ __forceinline__ int32_t card_off(int card, int V) {
  return card >= 0 ? (int32_t)((uint32_t)card * (uint32_t)V * 4u) : (int32_t)0x80000000u;
}

// LDS-DMAs are written as inline asm (kl_dwo2_kernel): the compiler's wait insertion treats a
// pending LDS-DMA as a possible writer of every later LDS read (no alias information here) and puts
// a vmcnt(0) before unrelated LDS reads, draining the very DMAs meant to run under them.  Invisible to it, they only make its own counted waits
// stricter than needed (it counts fewer younger accesses than there are); the slots' own waits
// are the explicit ones in the kernel.
typedef __attribute__((ext_vector_type(4))) int32_t v4i;
__device__ __forceinline__ v4i sgpr_rsrc(const void *base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  return v4i{__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a), __builtin_amdgcn_readfirstlane((int32_t)(a >> 32) & 0xFFFF),
             __builtin_amdgcn_readfirstlane((int32_t)bytes), 0x00020000};
}
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_void *)p);
}
// lane L: 'size' bytes at rsrc + voff + soff -> LDS lds + size L.  (M0 is reserved — not a
// clobber the compiler takes — and nothing else in these kernels reads it: checked in the ISA.)
template <int SIZE, int CPOL>
__device__ __forceinline__ void dma_asm(const v4i &rs, uint32_t voff, uint32_t soff, uint32_t lds) {
  static_assert(SIZE == 16 || SIZE == 4, "dwordx4 / dword");
  if constexpr (SIZE == 16 && CPOL == KL_CPOL_NT)
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, %3 offen nt lds" ::"v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
  else if constexpr (SIZE == 16)
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds" ::"v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
  else
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dword %0, %1, %3 offen lds" ::"v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
}

template <int D, bool FIX, int CPOL = 0, bool DW = true, bool WS = false>
__device__ __forceinline__ void kl_slice(const KlP &p, const int sl, bf16_t *Wt, MainSmem<kl_nb<D>()> &sm) {
  constexpr int NB = kl_nb<D>(), NJ = NB / 32;
  constexpr int CHB = TR / 8;
  // (w through readfirstlane: wave-uniform to the compiler, so the per-wave conditions below are
  // scalar branches and the counted waits of each path stay exact)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), half = lane >> 5;
  const int n0 = sl * NB;
  const int V = p.V;
  KL_PROBE(0);
  load_wo_slice<D>(p.Wo, V, n0, Wt);
  float bias[NJ], cs[NJ];
  bool valid[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int gc = n0 + j * 32 + (lane & 31);
    valid[j] = gc < V;
    bias[j] = valid[j] ? p.bo[gc] : 0.f;
    cs[j] = 0.f;
  }
  float klsum = 0.f, klc = 0.f;   // klc: slice 0 adds each live row's sum_j t ln t once
  bool dead = false;
  // M~ rows and dZ through buffer descriptors: a 32-bit byte offset per access instead of a 64-bit
  // address (M~ < 4 GB at |V| <= 32k; dZ rows x V x 2 B < 4 GB)
  // (out-of-range offsets — padding rows, columns past V — read 0 / drop the store: no branches)
  const __amdgpu_buffer_rsrc_t mt_rs = __builtin_amdgcn_make_buffer_rsrc((void *)p.Mt, (short)0, p.mt_bytes, 0x00020000);  // < 2^31
  const __amdgpu_buffer_rsrc_t dz_rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)p.dZ, (short)0, (uint32_t)p.rows * (uint32_t)V * 2u, 0x00020000);
  const float scale = p.scale;
  constexpr int ND2 = (D + 255) / 256;   // phase 2's d tiles of wave w: 32w .. (and 32(w + 8) .. at d = 512)
  // PF (the main pass with dWo done elsewhere: many row tiles, nothing of phase 2 live): the next
  // row block's A fragments load right after this block's logits MFMAs, so their L2 / MALL round
  // trip runs under this block's epilogue instead of heading the next logits phase (tools/micro/
  // kl_probe_full.hip: ~5 of the ~12 us per 256-row pass were logits waiting on their fragments)
  constexpr bool PF = !FIX && !DW && D <= 256;
  // WSX (PF with M~ in registers; the launcher checks |V| % 8 == 0 and the offsets' range): dZ leaves
  // through the free dZ^T LDS as 16-B row stores.  The accumulator layout gives a lane one column
  // of 16 rows, so a direct store writes 2 B per lane — 48 buffer_store_short per lane and pass,
  // issue-bound (the pass without its dZ stores ran ~20 % faster, kl_probe_full KL_DIAG_NOSTORE).
  // Instead adjacent lanes pair their bf16 values by one DPP swap into row-major dwords, the wave
  // writes its [32][96] tile to a private LDS image (208-B pitch: no bank conflicts between the
  // half-waves' rows), reads it back as 16-B row chunks and stores 6 x 16 B per lane.
  constexpr bool WSX = WS && PF;
  constexpr int WS_PITCH = 52;   // dwords per image row (96 bf16 + 8 pad)
  uint32_t *const zimg = reinterpret_cast<uint32_t *>(sm.Zt) + w * (32 * WS_PITCH);
  static_assert(!WSX || 8 * 32 * WS_PITCH * 4 <= (int)sizeof(sm.Zt), "WS: the images fit the dZ^T tile");
  // all A fragments first in the memory queue, then M~ (d = 512: a ring of 16; PF: the next block's
  // first 8 under the epilogue, the other 8 refilled during the MFMAs — 16 would spill)
  LFrag<D, PF ? 8 : (D / 16 < 16 ? D / 16 : 16)> lf;
  bool lf_ready = false;


  for (int t0 = 0; t0 < p.rows; t0 += TR) {
    const int nt = min(TR, p.rows - t0);
    auto rowoff = [&](int i) -> uint32_t { return (uint32_t)sm.card[i]; };   // tile row i's M~ offset
    lds_barrier();  // previous tile's phase 2 done with Zt / rs
    for (int i = tid; i < nt; i += NTH) {
      float4 st = p.rowstat[t0 + i];
      if constexpr (FIX) {  // .z <- delta of the row: the sum of its slices' partials, in order
        float dl = 0.f;
        const float *pd = p.part_d + (int64_t)(t0 + i) * p.nsl;
        for (int s = 0; s < p.nsl; ++s) dl += pd[s];
        st.z = dl;
      }
      sm.rs[i] = st;
      const int card = p.reg_idx[t0 + i];
      if (!FIX && sl == 0 && card >= 0) klc += st.w;
      sm.card[i] = card_off(card, V);
    }
    lds_barrier();
    KL_PROBE(1);
    // ---- phase 1: two passes of 8 waves x 32 rows
#pragma unroll 1
    for (int ps = 0; ps < 2; ++ps) {
      const int rb = ps * 256 + w * 32;  // tile-local first row of the wave
      if (rb >= nt) continue;            // wave-uniform
      // row byte offsets into M~ (card * V * 4), or a sentinel past the buffer's range for
      // padding rows: their loads return 0 without touching memory.  Loads are unconditional
      // (a conditional load becomes a branch with a wait per load) and all of the pass's are
      // issued before its logits, so their HBM latency runs under the MFMAs.
      uint32_t roff[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) roff[r] = rowoff(rb + acc_row(r, lane));
      uint32_t zrow = (uint32_t)((t0 + rb + 4 * half) * V + n0 + (lane & 31));
      asm volatile("" : "+v"(zrow));  // per-pass base of the dZ stores (no hoisted 64-bit addresses)
      if (!PF || !lf_ready) logits_load(p, (p.row0 + t0 + rb) / 32, lf);
      // PF: this wave's next row block — pass 1 of this tile, or pass 0 of the next (wave-uniform)
      int t1 = 0, rb1 = 0;
      bool nxt = false;
      if constexpr (PF) {
        t1 = ps == 0 && 256 + w * 32 < nt ? t0 : t0 + TR;
        rb1 = t1 == t0 ? 256 + w * 32 : w * 32;
        nxt = t1 < p.rows && rb1 < min(TR, p.rows - t1);
      }
      float tv[NJ][16];
      if constexpr (!FIX) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const uint32_t gc4 = 4u * (uint32_t)(n0 + j * 32 + (lane & 31));
#pragma unroll
          for (int r = 0; r < 16; ++r)
            tv[j][r] = KL_DIAG_NOMT ? (float)(r + j) * 1e-3f
                                    : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mt_rs, roff[r] + gc4, 0, CPOL));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x16_t acc[NJ];
      logits_mfma(Wt, lf, bias, acc);
      if constexpr (PF) {
        lf_ready = nxt;
        if (lf_ready) logits_load(p, (p.row0 + t1 + rb1) / 32, lf);
        __builtin_amdgcn_sched_barrier(0);
      }
      KL_PROBE(2 + 2 * ps);
      bool deadp = false;   // an element of this pass has p < 1e-7
      float mn = 1.f;       // (fast path) the smallest p of the lane's elements
      // wave-uniform: every row of the wave is a real regulariser row (no padding)
      bool rows_ok = true;
#pragma unroll
      for (int r = 0; r < 16; ++r) rows_ok &= roff[r] < 0x80000000u;
      rows_ok = __ballot(!rows_ok) == 0ull;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = j * 32 + (lane & 31);
        uint16_t tt[16];
        // row stats re-read per column tile (an opaque base): held across the three tiles they
        // cost 64 VGPRs, LDS has the bandwidth
        int rsofs = 0;
        asm volatile("" : "+v"(rsofs));
        const float4 *rsp = sm.rs + rsofs;
        // {m + ln s, S (FIX: delta)} of tile row i
        auto rstat = [&](int i) -> float2 {
          const float4 q = rsp[i];
          return make_float2(q.x, q.z);
        };
        // the common case — all rows real, all 32 columns inside V: no per-element masks, the
        // clip of q folded into one med3 (ln clip(p, 1e-7, 1) = med3(ln p, ln 1e-7, 0)), the
        // dead-element test as a running min of p
        const bool fast = !FIX && rows_ok && __ballot(!valid[j]) == 0ull;
        // WSX: rows r - 1, r (r odd) of columns c, c ^ 1 -> one dword per lane, right after row r's
        // value (so no more than a pair of them is live)
        auto ws_pair = [&](int r, uint32_t lo, uint32_t hi) {
          if constexpr (WSX) {
            const bool odd = lane & 1;
            const uint32_t give = odd ? lo : hi;
            const uint32_t got = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)give, 0xB1, 0xF, 0xF, false);   // lane ^ 1
            const uint32_t dw = odd ? (got | (hi << 16)) : (lo | (got << 16));
            zimg[(acc_row(r - 1, lane) + (odd ? 1 : 0)) * WS_PITCH + j * 16 + ((lane & 31) >> 1)] = dw;
          }
        };
        if (fast) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float2 st = rstat(rb + acc_row(r, lane));
            const float lp = acc[j][r] - st.x;  // ln p = z - (m + ln s)
            const float pr = __builtin_amdgcn_exp2f(lp * LOG2E);
            const float tc = __builtin_amdgcn_fmed3f(tv[j][r], PMIN, 1.f);
            klsum = fmaf(-tc, __builtin_amdgcn_fmed3f(lp, LN_PMIN, 0.f), klsum);   // (+ t ln t: rowstat.w)
            mn = fminf(mn, pr);
            // (the product as fma(.., +0): a rounded value the column sum below cannot contract into
            // an fma with it — the same bits whichever way the compiler shapes the code, MS or not)
            const float dzf = fmaf(scale, fmaf(pr, st.y, pr >= PMIN ? -tc : 0.f), 0.f);
            const uint16_t zb = bf16_bits(dzf);
            tt[r] = zb;
            cs[j] += dzf;  // the bias gradient sums the fp32 dz
            // the lane part of the offset in a VGPR, the row part (r) as the scalar soffset
            if constexpr (!WSX && !KL_DIAG_NOSTORE)
              __builtin_amdgcn_raw_buffer_store_b16(zb, dz_rs, 2u * (zrow + (uint32_t)(j * 32)),
                                                    2u * (uint32_t)(((r & 3) + 8 * (r >> 2)) * V), CPOL);
            if (r & 1) ws_pair(r, tt[r - 1], zb);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int lr = rb + acc_row(r, lane);
            const float2 st = rstat(lr);
            const bool live_row = roff[r] < 0x80000000u && valid[j];
            const float lp = acc[j][r] - st.x;  // ln p = z - (m + ln s)
            const float pr = __builtin_amdgcn_exp2f(lp * LOG2E);
            const bool live = pr >= PMIN;
            float dz;
            if constexpr (!FIX) {
              const float tc = __builtin_amdgcn_fmed3f(tv[j][r], PMIN, 1.f);
              const float lq = live ? fminf(lp, 0.f) : LN_PMIN;  // ln clip(p, 1e-7, 1)
              const float term = -tc * lq;   // (the row's sum of t ln t: rowstat.w, added once)
              klsum += live_row ? term : 0.f;
              deadp |= live_row && !live;
              dz = live_row ? fmaf(scale, fmaf(pr, st.y, live ? -tc : 0.f), 0.f) : 0.f;
            } else {
              dz = live_row ? -scale * pr * st.y : 0.f;  // st.y = delta
            }
            const uint32_t zoff = 2u * (zrow + (uint32_t)(((r & 3) + 8 * (r >> 2)) * V + j * 32));
            uint16_t zb;
            if constexpr (FIX) {
              const float old = valid[j] ? bf2f(p.dZ[zoff / 2]) : 0.f;
              zb = bf16_bits(old + dz);
              dz = __uint_as_float((uint32_t)zb << 16) - old;  // the change actually applied
              tt[r] = bf16_bits(dz);
              cs[j] += __uint_as_float((uint32_t)tt[r] << 16);
            } else {
              zb = bf16_bits(dz);
              tt[r] = zb;
              cs[j] += dz;
            }
            if (!WSX && valid[j]) __builtin_amdgcn_raw_buffer_store_b16(zb, dz_rs, zoff, 0, CPOL);
            if constexpr (!FIX)
              if (r & 1) ws_pair(r, tt[r - 1], zb);
          }
        }
        if constexpr (DW) {
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<uint2 *>(sm.Zt + sw_off(col, rb + 8 * g + 4 * half, CHB)) =
                *reinterpret_cast<const uint2 *>(&tt[4 * g]);
        }
      }
      deadp |= mn < PMIN;
      if constexpr (WSX) {   // the wave's [32][96] dZ image -> 6 x 16 B per lane (chunks past V dropped)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int q = lane + 64 * u, row = q / 12, ch = q % 12;
          const v4u x = *reinterpret_cast<const v4u *>(zimg + row * WS_PITCH + ch * 4);
          const uint32_t off = n0 + 8 * ch < V ? 2u * ((uint32_t)(t0 + rb + row) * (uint32_t)V + (uint32_t)(n0 + 8 * ch))
                                               : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b128(x, dz_rs, off, 0, KL_ZST_CPOL < 0 ? CPOL : KL_ZST_CPOL);
        }
      }

      if constexpr (!FIX) {
        // the exact-clip delta partial of each row over this slice: sum of its targets where
        // p < 1e-7 (rare: zero unless the wave saw such an element); read by the fix kernel
        float red = 0.f;
        if (__ballot(deadp) != 0ull) {
          // per column tile (one tile's targets live at a time), the same order of additions
          float dl[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) dl[r] = 0.f;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            float tj[16];
            const uint32_t gc4 = 4u * (uint32_t)(n0 + j * 32 + (lane & 31));
#pragma unroll
            for (int r = 0; r < 16; ++r) tj[r] = tv[j][r];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float st_x = sm.rs[rb + acc_row(r, lane)].x;
              const float pr = __builtin_amdgcn_exp2f((acc[j][r] - st_x) * LOG2E);
              const bool live_row = roff[r] < 0x80000000u && valid[j];
              dl[r] += live_row && !(pr >= PMIN) ? __builtin_amdgcn_fmed3f(tj[r], PMIN, 1.f) : 0.f;
            }
          }
          red = rs16<false>(dl);
        }
        if ((lane & 1) == 0)
          p.part_d[(int64_t)(t0 + rb + acc_row((lane >> 1) & 15, lane)) * p.nsl + sl] = red;
      }
      KL_PROBE(3 + 2 * ps);
      if constexpr (!FIX) dead |= deadp;
    }
    if constexpr (!DW) continue;   // dWo by kl_dwo_kernel from the stored dZ
    lds_barrier();
    KL_PROBE(6);
    // ---- phase 2: dWo[d][NB] (+)= D3^T[d][tile rows] dZ[tile rows][NB] (wave w: d rows 32w..).
    // A fresh accumulator per tile, added into gW (the block's slice stays L2-resident between
    // tiles): nothing of phase 2 is live across phase 1's epilogue.
#pragma unroll
    for (int dt = 0; dt < ND2; ++dt) {
      const int wt = w + 8 * dt;   // this d tile (rows 32 wt .. of dWo)
      if (wt * 32 >= D) break;
      f32x16_t acc2[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[j][r] = 0.f;
      // K = the tile's rows (a multiple of 32) in chunks of 32 (two 16-row fragments), a ring of
      // P2 chunks in flight (the loads come from L2: one chunk's 6 MFMAs cannot cover one latency)
      constexpr int P2 = 6;
      const int nc = nt / 32;
      const int j0 = (p.row0 + t0) / 16;
      const bf16_t *arow = p.D3tp + ((int64_t)wt * (p.ldt / 16) * 64 + lane) * 8 + (int64_t)j0 * 512;
      bf16x8_t ring[P2][2];
#pragma unroll
      for (int q = 0; q < P2; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) ring[q][h] = *reinterpret_cast<const bf16x8_t *>(arow + (2 * min(q, nc - 1) + h) * 512);
      for (int c0 = 0; c0 < nc; c0 += P2) {
#pragma unroll
        for (int q = 0; q < P2; ++q) {
          const int c = c0 + q;
          if (c < nc) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int j = 0; j < NJ; ++j) {
                const bf16x8_t b = frag(sm.Zt, sw_off(j * 32 + (lane & 31), c * 32 + h * 16 + 8 * half, CHB));
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ring[q][h], b, acc2[j], 0, 0, 0);
              }
            const int cn = min(c + P2, nc - 1);
#pragma unroll
            for (int h = 0; h < 2; ++h) ring[q][h] = *reinterpret_cast<const bf16x8_t *>(arow + (2 * cn + h) * 512);
          }
        }
      }
      const bool first = !FIX && t0 == 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int gc = n0 + j * 32 + (lane & 31);
        if (gc < V) {
          uint32_t g0 = (uint32_t)((wt * 32 + 4 * half) * V + gc);
          asm volatile("" : "+v"(g0));  // opaque per tile: keeps 48 row addresses from being hoisted
          // the tile's 16 partial sums of this column are added to gW with 8 loads in flight at
          // a time (a load-add-store per element serialised 48 round trips per tile: the
          // full-mode regulariser walks 43 tiles per slice).  (Measured and dropped: all 48 loads
          // issued before the MFMA chain — the extra live registers spilled, 1,590 -> 2,040 us
          // per block in full mode.)
#pragma unroll
          for (int h8 = 0; h8 < 16; h8 += 8) {  // two groups of 8 loads in flight (registers)
            float old[8];
            if (!first) {
#pragma unroll
              for (int r = 0; r < 8; ++r) old[r] = p.gW[g0 + (uint32_t)((((h8 + r) & 3) + 8 * ((h8 + r) >> 2)) * V)];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r)
              p.gW[g0 + (uint32_t)((((h8 + r) & 3) + 8 * ((h8 + r) >> 2)) * V)] =
                  first ? acc2[j][h8 + r] : old[r] + acc2[j][h8 + r];
          }
        }
      }
    }
  }

  KL_PROBE(7);
  // ---- epilogue: dbo, loss partial, the fix flag
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float c2 = cs[j] + __shfl_xor(cs[j], 32);
    if (half == 0) sm.red_cs[w][j * 32 + (lane & 31)] = c2;
  }
  if constexpr (!FIX) {
    if (__ballot(dead) != 0ull && lane == 0)
      __hip_atomic_fetch_or(p.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    klsum += klc;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) klsum += __shfl_xor(klsum, off);
    if (lane == 0) sm.red_loss[w] = (double)klsum;
  }
  lds_barrier();
  if (tid < NB && n0 + tid < V) {
    float g = 0.f;
    for (int i = 0; i < NTH / 64; ++i) g += sm.red_cs[i][tid];
    if constexpr (FIX)
      p.gb[n0 + tid] += g;
    else
      p.gb[n0 + tid] = g;
  }
  if constexpr (!FIX) {
    if (tid == 0) {
      double sum = 0.0;
      for (int i = 0; i < NTH / 64; ++i) sum += sm.red_loss[i];
      sm.lastflag = 0;
      if (!p.loss_out) {
        p.loss_partials[sl] = sum;
      } else {
        __hip_atomic_store(&p.loss_partials[sl], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t tk = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sm.lastflag = tk == gridDim.x - 1;
      }
    }
    if (p.loss_out) {
      __syncthreads();
      if (sm.lastflag) {
        double s2d = 0.0;
        for (int i = tid; i < (int)gridDim.x; i += NTH)
          s2d += __hip_atomic_load(&p.loss_partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s2d += __shfl_xor(s2d, off);
        if (lane == 0) sm.red_loss[w] = s2d;
        __syncthreads();
        if (tid == 0) {
          double tot = 0.0;
          for (int i = 0; i < NTH / 64; ++i) tot += sm.red_loss[i];
          p.loss_out[0] = tot * p.loss_scale;
          __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

template <int D, int CPOL, bool DW, bool WS = false>
__global__ __launch_bounds__(NTH) void kl_main_kernel(KlP p) {
  __shared__ __attribute__((aligned(16))) bf16_t Wt[kl_nb<D>() * D];
  __shared__ __attribute__((aligned(16))) MainSmem<kl_nb<D>()> sm;
  kl_slice<D, false, CPOL, DW, WS>(p, cc_slice_of_block(blockIdx.x, gridDim.x), Wt, sm);
}

// (Measured and dropped, round 6: the main pass with the MFMA operands swapped as in the stats
// kernels — a lane = one row: 16-B M~ loads, 16-B dZ row stores after permlane32 swaps, the row
// stats per lane, the bias by one MFMA against a ones fragment, the column sums reduce-scattered;
// correct, but full mode 2.78 against 2.23 ms/step and the sampled + KL step 280 against 275.5 us:
// a 16-B load or store of this layout touches 32 rows per wave instruction where the 4-B / 2-B
// accesses of kl_slice's layout touch 2.  Source at commit 997c871.)

// The exact-clip correction: a small persistent grid (FIXG blocks) that leaves at once when the
// step saw no p < 1e-7, and otherwise walks the slices.
constexpr int FIXG = 64;
template <int D, bool DW>
__global__ __launch_bounds__(NTH) void kl_fix_kernel(KlP p) {
  __shared__ __attribute__((aligned(16))) bf16_t Wt[kl_nb<D>() * D];
  __shared__ __attribute__((aligned(16))) MainSmem<kl_nb<D>()> sm;
  if (__hip_atomic_load(p.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  for (int sl = blockIdx.x; sl < p.nsl; sl += gridDim.x) {
    kl_slice<D, true, 0, DW>(p, sl, Wt, sm);
    __syncthreads();  // LDS reuse by the next slice
  }
}

// ---------------------------------------------------------------- dWo from the stored dZ
// Many row tiles (the full-mode regulariser: all |V| identity rows): dWo[d][V] = D3^T[d][rows]
// dZ[rows][V] as its own product, after the main (and fix) pass stored the final bf16 dZ — the
// product the main pass folded into every row tile as a per-tile read-modify-write of the block's
// slice (~16 of ~38 us per 512-row tile, tools/micro/kl_probe_full.hip).  One block per 96-column
// slice and 256 rows of d owns its dWo tile over the whole K = rows reduction in registers: no
// partial sums, one store per element, the same MFMA k order for every element (deterministic).
// dZ chunks of DW_KC rows x 96 columns are staged global -> registers -> LDS as raw rows (each
// thread 3 x 16 B per chunk, loaded three chunks and written one chunk ahead of its use; two LDS
// stages, one barrier per chunk); B fragments by ds_read_b64_tr_b16 (column n, 4 consecutive rows per read; the 192-B rows
// put 4 consecutive rows on disjoint banks); A fragments from the packed D3^T image (1 KB per wave
// load), one chunk ahead in registers.  Wave w owns 32 rows of d x the 3 column tiles.
// (Staged by LDS-DMA instead, the compiler waits for every outstanding copy — vmcnt(0) — before
// each chunk's LDS reads, so nothing stays in flight.)
constexpr int DW_NB = 96, DW_KC = 128;
// build knob (A/B): kl_dwo_kernel's B fragments one k step ahead
#ifndef DWO_BPF
#define DWO_BPF 1
#endif
// dev diagnostics (tools/micro/dwo_diag.hip; 0 in the library): 1 no MFMA, 2 no B reads, 4 no dZ
// loads, 8 no A loads
#ifndef DWO_DIAG
#define DWO_DIAG 0
#endif
template <int D, bool V8>
__global__ __launch_bounds__(NTH) void kl_dwo_kernel(KlP p) {
  constexpr int NB = DW_NB, NJ = NB / 32, KC = DW_KC, KS = KC / 16;
  constexpr int PPR = NB / 8;                    // 16-B pieces per chunk row
  constexpr int NPC = KC * PPR / NTH;            // pieces per thread per chunk
  static_assert(KC * PPR % NTH == 0, "kl_dwo_kernel: whole pieces per thread");
  typedef short v4s __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) bf16_t Zs[2][KC * NB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5;
  const int n0 = blockIdx.x * NB, V = p.V;
  const int wt = blockIdx.y * 8 + w;              // this wave's 32 rows of d
  const bool active = wt * 32 < D;                // (d = 128: waves 4-7 only copy)
  const int nch = (p.rows + KC - 1) / KC;
  const __amdgpu_buffer_rsrc_t zr =
      __builtin_amdgcn_make_buffer_rsrc((void *)p.dZ, (short)0, (uint32_t)p.rows * (uint32_t)V * 2u, 0x00020000);
  // piece q = tid + NTH u of chunk c = (row q / PPR, 16 B e = q % PPR); rows past `rows` read 0
  // (beyond the descriptor's range), columns past V read the next row (finite; not stored)
  // two register sets: chunk c's pieces are loaded at iteration c - 3 and written to LDS at
  // iteration c - 1, two chunk times of lead (one chunk time, ~0.7 us, left the HBM latency exposed:
  // 24 KB in flight per CU, ~2.7 TB/s)
  v4u stg0[NPC], stg1[NPC];
  auto gload = [&](v4u (&stg)[NPC], int c) {
    if constexpr (DWO_DIAG & 4) return;
#pragma unroll
    for (int u = 0; u < NPC; ++u) {
      const int q = tid + NTH * u, r = q / PPR, e = q % PPR;
      const uint32_t off = (uint32_t)(((c * KC + r) * V + n0) * 2 + e * 16);
      if constexpr (V8) {
        stg[u] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(zr, off, 0, 0));
      } else {   // 4-B aligned rows (V even)
#pragma unroll
        for (int h = 0; h < 4; ++h) stg[u][h] = __builtin_amdgcn_raw_buffer_load_b32(zr, off + 4 * h, 0, 0);
      }
    }
  };
  auto swrite = [&](const v4u (&stg)[NPC], int st) {
#pragma unroll
    for (int u = 0; u < NPC; ++u) *reinterpret_cast<v4u *>(Zs[st] + (tid + NTH * u) * 8) = stg[u];
  };
  // A fragment (k step ks of chunk c): packed D3^T, clamped to the last k step (its dZ rows are 0)
  const bf16_t *abase = p.D3tp + ((int64_t)min(wt, D / 32 - 1) * (p.ldt / 16) * 64 + lane) * 8;
  const int k0 = p.row0 / 16, klast = (p.row0 + p.rows) / 16 - 1;
  auto load_a = [&](bf16x8_t (&dst)[KS], int c) {
    if constexpr (DWO_DIAG & 8) return;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      dst[ks] = *reinterpret_cast<const bf16x8_t *>(abase + (int64_t)min(k0 + c * KS + ks, klast) * 512);
  };
  f32x16_t acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  bf16x8_t af[2][KS];
  // (issue order as in the steady state — chunk c + 1's pieces, chunk c's A fragments, chunk c + 2's
  // pieces — so the compiler's counted waits at the loop head, merged over entry and back edge, are
  // the steady state's and not a drain to the newest chunk)
  gload(stg0, 0);
  swrite(stg0, 0);
  gload(stg1, 1);
  load_a(af[0], 0);
  gload(stg0, 2);
  lds_barrier();
  // chunk c: stage st = c & 1.  Write chunk c + 1 (register set (c + 1) & 1, loaded two chunks ago)
  // into the other stage, load chunk c + 3 into that set and chunk c + 1's A fragments, multiply
  // chunk c, barrier.
  auto body = [&](bf16x8_t (&cur)[KS], bf16x8_t (&nxt)[KS], v4u (&sw)[NPC], int c, const int st) {
    // unconditional (past the last chunk: zeros / clamped fragments, never read) so the compiler's
    // counted waits for `cur` and the staged pieces stay exact (a branch merges them to the minimum)
    // (A before the pieces: waiting for chunk c + 1's A fragments — vmcnt counts in issue order —
    // must not wait for chunk c + 3's pieces)
    swrite(sw, st ^ 1);
    load_a(nxt, c + 1);
    gload(sw, c + 3);
    if (active) {
      const bf16_t *Zc = Zs[st];
      auto bfrag = [&](int ks, int j) {
        if constexpr (DWO_DIAG & 2) return cur[(ks + j) % KS];
        const bf16_t *tb = Zc + (ks * 16 + 8 * half + ((lane >> 2) & 3)) * NB + j * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)tb);
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)(tb + 4 * NB));
        return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      };
      if constexpr (DWO_BPF) {
        // B fragments one k step ahead (two register sets): the k step's MFMAs wait on reads issued
        // a whole step earlier, not on the ones just before them
        bf16x8_t bq[2][NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bq[0][j] = bfrag(0, j);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if (ks + 1 < KS) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) bq[(ks + 1) & 1][j] = bfrag(ks + 1, j);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            if constexpr (DWO_DIAG & 1) {
              acc[j][0] += __builtin_bit_cast(float, __builtin_shufflevector(bq[ks & 1][j], bq[ks & 1][j], 0, 1));
              acc[j][1] += __builtin_bit_cast(float, __builtin_shufflevector(cur[ks], cur[ks], 0, 1));
            } else {
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[ks], bq[ks & 1][j], acc[j], 0, 0, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[ks], bfrag(ks, j), acc[j], 0, 0, 0);
      }
    }
    lds_barrier();   // chunk c + 1 written; chunk c read (its stage is rewritten next)
  };
  int c = 0;
  for (; c + 1 < nch; c += 2) {
    body(af[0], af[1], stg1, c, 0);
    body(af[1], af[0], stg0, c + 1, 1);
  }
  if (c < nch) body(af[0], af[1], stg1, c, 0);
  if (!active) return;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int gc = n0 + j * 32 + (lane & 31);
    if (gc < V) {
#pragma unroll
      for (int r = 0; r < 16; ++r) p.gW[(int64_t)(wt * 32 + acc_row(r, lane)) * V + gc] = acc[j][r];
    }
  }
}

// ---- dWo in wide slices (the default for d = 256, |V| % 8 == 0): kl_dwo_kernel spends its time
// on the per-CU operand streams, not on the MFMAs: every 96-column block re-reads the whole packed
// D3^T (11 MB at the full-mode shape — 2.7x the block's dZ bytes) and each of its 8 waves reads the
// whole dZ chunk from LDS (tools/micro/dwo_diag.hip: the D3^T loads alone 134 us of its 345).
// Here a block owns a 192-column slice and HALF of the rows (K split in two: 2 x 115 blocks), eight
// waves (two per SIMD) of 32 rows of d x all 192 columns (6 accumulator tiles): per column, half
// the D3^T bytes of kl_dwo_kernel.  dZ chunks of 128 rows x 192 columns (48 KB) are copied
// global -> LDS by 16-B LDS-DMA (non-temporal: read once) two chunks ahead of use in a ring of
// three stages; A fragments (8 k steps per wave) load one chunk ahead into registers.
// Measured alone at the full-mode shape (tools/micro/dwo_diag.hip, r05z): 242 us + 13 us for the
// halves' sum vs kl_dwo_kernel's 343; four waves of 64 rows (accumulators in AGPRs, one wave per
// SIMD) 273, default cache policy on the copies 264, copies issued before the A loads (one chunk
// of effective lead: the in-order wait for A(c) also waited for DMA(c + 1)) 294.  Both streams are inline asm with counted waits written here (the
// compiler's own waits would count only what it sees; see dma_asm), in one fixed per-wave issue
// order — A(c + 1), DMA(c + 2) per chunk c — so the counts are constants.  The LDS rows (384 B)
// are stored with 16-B pieces XOR 4 on rows with bit 1 set (the DMA picks the source piece), which
// puts the four rows of a ds_read_b64_tr_b16 lane group on disjoint banks.  The first half's
// partial tile goes to the workspace, the second's to gW, and kl_dwo2_sum_kernel adds them (an
// arrival ticket per slice with the second block adding instead cost ~100 us: the agent-scope
// fences' L2 write-back / invalidate under the still-streaming blocks).
#ifndef CCREC_DWO2
#define CCREC_DWO2 1   // build knob (A/B builds): 0 = dWo by the 96-column kernels always
#endif
// dev diagnostics (tools/micro/dwo_diag.hip; 0 in the library): 2 no MFMA, 4 no dZ DMA, 8 no A
// loads
#ifndef DW2_DIAG
#define DW2_DIAG 0
#endif
#ifndef DW2_CPOL
#define DW2_CPOL KL_CPOL_NT   // build knob: the dZ copies' cache policy (0: default)
#endif
#ifndef DW2_WAVES
#define DW2_WAVES 8   // build knob: 8 waves of 32 rows of d (two per SIMD) or 4 of 64 (one per SIMD)
#endif
constexpr int DW2_NB = 192, DW2_KC = 128, DW2_NS = 3, DW2_NT = 64 * DW2_WAVES, DW2_SPLIT = 2;
constexpr int DW2_STAGE = DW2_KC * DW2_NB * 2;          // 48 KB
constexpr int DW2_LDS = DW2_NS * DW2_STAGE;             // 144 KB

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// 16 B per lane into registers, invisible to the compiler's counters: the caller waits (vm_wait)
// and then re-defines the registers through an empty asm before any use
__device__ __forceinline__ v4u a_load(const v4i &rs, uint32_t voff, uint32_t soff) {
  v4u r;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(r) : "v"(voff), "s"(rs), "s"(soff));
  return r;
}

template <int D>
__global__ __launch_bounds__(DW2_NT) void kl_dwo2_kernel(KlP p) {
  constexpr int NW = DW2_NT / 64, NBD = D / 32 / NW;    // waves; 32-row bands of d per wave
  static_assert(D == 256 && NBD * NW * 32 == D, "d = 256 over the waves");
  constexpr int NB = DW2_NB, NJ = NB / 32, KC = DW2_KC, KS = KC / 16, NS = DW2_NS;
  constexpr int PPR = NB / 8;                            // 16-B pieces per chunk row
  constexpr int NPW = DW2_STAGE / 1024 / NW;             // DMA instructions per wave per chunk
  constexpr int NA = NBD * KS;                           // A loads per wave per chunk
  static_assert(DW2_STAGE % (1024 * NW) == 0 && NPW + NA + NPW <= 63, "whole DMA instructions; vmcnt range");
  typedef short v4s __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(1024))) char dw2mem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), half = lane >> 5;
  const int sl = blockIdx.x, kh = blockIdx.y;
  const int n0 = sl * NB, V = p.V;
  const int nall = (p.rows + KC - 1) / KC;
  const int cb = nall * kh / DW2_SPLIT, nch = nall * (kh + 1) / DW2_SPLIT - cb;
  const v4i zr = sgpr_rsrc(p.dZ, (uint32_t)p.rows * (uint32_t)V * 2u);
  const v4i ar = sgpr_rsrc(p.D3tp, (uint32_t)p.ldt * (uint32_t)D * 2u);
  // DMA instruction t of this wave: LDS bytes [1024 (NPW w + t), ..) of the stage; lane L's 16 B are
  // stage piece s = 64 (NPW w + t) + L = row s / PPR, position s % PPR, holding dZ piece
  // position ^ 4 (row >> 1 & 1) of that row.  Columns past V read the next row / past the range
  // (finite or 0; never stored), chunks past this half's end the sentinel (zeros, no traffic).
  uint32_t vo[NPW];
#pragma unroll
  for (int t = 0; t < NPW; ++t) {
    const int s = (NPW * w + t) * 64 + lane, r = s / PPR, e = (s % PPR) ^ (4 * ((r >> 1) & 1));
    vo[t] = (uint32_t)(r * V + n0) * 2u + 16u * (uint32_t)e;
  }
  const uint32_t lbase = lds_addr(dw2mem) + 1024u * (uint32_t)(NPW * w);
  auto dma = [&](int c) {
    if constexpr (DW2_DIAG & 4) return;
    const uint32_t so = c < nch ? (uint32_t)(cb + c) * (uint32_t)KC * (uint32_t)V * 2u : 0x80000000u;
    const uint32_t base = lbase + (uint32_t)(c % NS) * (uint32_t)DW2_STAGE;
#pragma unroll
    for (int t = 0; t < NPW; ++t) dma_asm<16, DW2_CPOL>(zr, vo[t], so, base + 1024u * t);
  };
  // A fragment (band b, k step kk): the packed D3^T's 1-KB fragment (band NBD w + b, kk)
  uint32_t va[NBD];
#pragma unroll
  for (int b = 0; b < NBD; ++b) va[b] = ((uint32_t)(NBD * w + b) * (uint32_t)(p.ldt / 16) * 64u + (uint32_t)lane) * 16u;
  const int k0 = p.row0 / 16, klast = (p.row0 + p.rows) / 16 - 1;
  auto aload = [&](v4u (&dst)[NBD][KS], int c) {   // (c past the end: clamped, never used)
    if constexpr (DW2_DIAG & 8) return;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint32_t so = (uint32_t)min(k0 + (cb + c) * KS + ks, klast) * 1024u;
#pragma unroll
      for (int b = 0; b < NBD; ++b) dst[b][ks] = a_load(ar, va[b], so);
    }
  };
  f32x16_t acc[NBD][NJ];
#pragma unroll
  for (int b = 0; b < NBD; ++b)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[b][j][r] = 0.f;
  v4u af[2][NBD][KS];
  // (a load's destination must stay allocated until its wait: a dead result register reused for
  // something else would be overwritten when the load lands — hence no dummy loads, and every
  // set kept live to the final wait)
  dma(0);
  aload(af[0], 0);
  dma(1);
  // B fragment (k step ks, column tile j) of a stage: rows ks 16 + 8 half + (lane >> 2 & 3) (+ 4),
  // 4 columns at j 32 + 16 (lane >> 4 & 1) + 4 (lane & 3), XOR 32 on rows with bit 1 set (= lane
  // bit 3): column tile j ^ 1 there, i.e. + 32 for even j and - 32 for odd j
  const int sw = 32 * ((lane >> 3) & 1);
  const int boff0 = (8 * half + ((lane >> 2) & 3)) * NB + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const int boff[2] = {boff0 + sw, boff0 - sw};
  // per chunk c: A(c + 1), then DMA(c + 2) — the wait for A(c) does not wait for DMA(c + 1), so
  // the copies keep two chunks of lead (DMA first, measured: one)
  auto body = [&](v4u (&cur)[NBD][KS], v4u (&nxt)[NBD][KS], int c) {
    vm_wait<NA + NPW>();        // own DMA(c) landed (younger: A(c), DMA(c + 1))
    lds_barrier();              // every wave's DMA(c) landed; stage (c - 1) % NS read by all
    aload(nxt, c + 1);
    dma(c + 2);
    vm_wait<NPW + NA + NPW>();  // A(c) landed (younger: DMA(c + 1), A(c + 1), DMA(c + 2))
#pragma unroll
    for (int b = 0; b < NBD; ++b)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(cur[b][ks]));
    const bf16_t *Zc = reinterpret_cast<const bf16_t *>(dw2mem + (c % NS) * DW2_STAGE);
    auto bfrag = [&](int ks, int j) {
      const bf16_t *tb = Zc + boff[j & 1] + ks * 16 * NB + j * 32;
      const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)tb);
      const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s *)(tb + 4 * NB));
      return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    bf16x8_t bq[2][NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bq[0][j] = bfrag(0, j);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) bq[(ks + 1) & 1][j] = bfrag(ks + 1, j);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int b = 0; b < NBD; ++b) {
        const bf16x8_t a = __builtin_bit_cast(bf16x8_t, cur[b][ks]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (DW2_DIAG & 2)
            acc[b][j][0] += __builtin_bit_cast(float, __builtin_shufflevector(bq[ks & 1][j], a, 0, 9));
          else
            acc[b][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq[ks & 1][j], acc[b][j], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int c = 0;
  for (; c + 1 < nch; c += 2) {
    body(af[0], af[1], c);
    body(af[1], af[0], c + 1);
  }
  if (c < nch) body(af[0], af[1], c);
  vm_wait<0>();   // the trailing (sentinel) DMAs land before the block's LDS is released
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int b = 0; b < NBD; ++b)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(af[u][b][ks]));   // (live to here: see above)
  // this half's partial: the first half into dw_part, the second into gW (kl_dwo2_sum_kernel adds)
  float *mine = kh == 0 ? p.dw_part : p.gW;
#pragma unroll
  for (int b = 0; b < NBD; ++b)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int gc = n0 + j * 32 + (lane & 31);
      if (gc < V) {
#pragma unroll
        for (int r = 0; r < 16; ++r) mine[(int64_t)(32 * (NBD * w + b) + acc_row(r, lane)) * V + gc] = acc[b][j][r];
      }
    }
}

// gW = dw_part + gW (the two row halves' partial dWo; n4 float4)
__global__ __launch_bounds__(256) void kl_dwo2_sum_kernel(const float4 *__restrict__ part, float4 *__restrict__ gw, int64_t n4) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 a = part[i], b = gw[i];
    gw[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
}

__global__ __launch_bounds__(256) void kl_tsum_kernel(const float *__restrict__ Mt, int V, float *__restrict__ tsum) {
  __shared__ float red[2][4];
  const float *row = Mt + (int64_t)blockIdx.x * V;
  float s = 0.f, c = 0.f;
  for (int j = threadIdx.x; j < V; j += 256) {
    const float t = __builtin_amdgcn_fmed3f(row[j], PMIN, 1.f);
    s += t;
    c = fmaf(t, __logf(t), c);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    c += __shfl_xor(c, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    reinterpret_cast<float2 *>(tsum)[blockIdx.x] =
        make_float2((red[0][0] + red[0][1]) + (red[0][2] + red[0][3]), (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
}

}  // namespace

extern "C" size_t cc_dec_kl_ws_size(int32_t rows, int32_t V) {
  const int64_t nsl = cdiv(V, NB_MIN);   // an upper bound over every d
  // (+ kl_dwo2_kernel's first-half partial dWo, d = 256, when rows take many tiles)
  const size_t dw2 = rows > TR ? (size_t)256 * V * sizeof(float) : 0;
  return (size_t)(3 * rows * nsl * sizeof(float) + rows * sizeof(float4) + 256 + rows * sizeof(float2)) + dw2;
}

extern "C" int32_t cc_dec_kl_blocks(int32_t V) { return (int32_t)cdiv(V, NB_MIN); }   // upper bound over d

extern "C" int cc_kl_tsum(const float *Mt, int32_t n, int32_t V, float *tsum, void *stream) {
  CC_REQUIRE(Mt && tsum && n >= 0 && V > 0, "cc_kl_tsum: args");
  if (n == 0) return CC_OK;
  hipLaunchKernelGGL(kl_tsum_kernel, dim3((unsigned)n), dim3(256), 0, as_stream(stream), Mt, V, tsum);
  CC_LAUNCH_CHECK("kl_tsum_kernel");
  return CC_OK;
}

extern "C" int cc_dec_softmax_kl_dw(const cc_dec_kl_args *a, void *stream) {
  CC_REQUIRE(a && a->D3p && a->D3tp && a->Wo && a->bo && a->Mt && a->tsum && a->reg_idx && a->dZ && a->gW &&
                 a->gb && a->loss_partials && a->ws,
             "cc_dec_softmax_kl_dw: null pointer");
  CC_REQUIRE(a->d == 128 || a->d == 256 || a->d == 512, "cc_dec_softmax_kl_dw: d must be 128, 256 or 512");
  const int NB = a->d <= 256 ? kl_nb<256>() : kl_nb<512>();
  CC_REQUIRE(a->rows > 0 && a->rows % 32 == 0, "cc_dec_softmax_kl_dw: rows must be a positive multiple of 32");
  CC_REQUIRE(a->row0 % 32 == 0 && a->ldt % 16 == 0 && a->ldt >= a->row0 + a->rows,
             "cc_dec_softmax_kl_dw: row0 % 32, ldt % 16, ldt >= row0 + rows");
  CC_REQUIRE(a->V > 0 && (!a->loss_out || a->ticket), "cc_dec_softmax_kl_dw: V / ticket");
  CC_REQUIRE(cdiv(a->V, NB) <= 64 * MRG, "cc_dec_softmax_kl_dw: V <= 49,152");
  CC_REQUIRE((((uintptr_t)a->D3p | (uintptr_t)a->D3tp | (uintptr_t)a->ws) & 15) == 0,
             "cc_dec_softmax_kl_dw: packed images and ws 16-B aligned");
  KlP p;
  p.d = a->d;
  p.V = a->V;
  p.rows = a->rows;
  p.ldt = a->ldt;
  p.row0 = a->row0;
  p.nsl = (int)cdiv(a->V, NB);
  p.D3p = (const bf16_t *)a->D3p;
  p.D3tp = (const bf16_t *)a->D3tp;
  p.Wo = (const bf16_t *)a->Wo;
  p.bo = a->bo;
  p.Mt = a->Mt;
  CC_REQUIRE(a->mt_bytes > 0 && a->mt_bytes <= 0x7FFFFFFFll && (int64_t)a->rows * a->V * 2 <= 0xFFFFFFFFll,
             "cc_dec_softmax_kl_dw: M~ extent below 2 GB and dZ below 4 GB (32-bit buffer offsets)");
  p.mt_bytes = (uint32_t)a->mt_bytes;
  CC_REQUIRE(a->mt_lo >= 0 && (int64_t)(a->mt_lo + 1) * a->V * 4 <= a->mt_bytes, "cc_dec_softmax_kl_dw: mt_lo");
  p.mt_lo = a->mt_lo;
  p.tsum = a->tsum;
  p.reg_idx = a->reg_idx;
  p.scale = a->scale;
  p.dZ = (bf16_t *)a->dZ;
  p.gW = a->gW;
  p.gb = a->gb;
  p.loss_partials = a->loss_partials;
  p.loss_out = a->loss_out;
  p.loss_scale = a->loss_scale;
  p.ticket = a->ticket;
  char *ws = (char *)a->ws;
  const int64_t pn = (int64_t)a->rows * p.nsl;
  p.rowstat = (float4 *)ws;
  p.part_m = (float *)(ws + a->rows * sizeof(float4));
  p.part_s = p.part_m + pn;
  p.part_d = p.part_s + pn;
  p.flag = (uint32_t *)(p.part_d + pn);
  p.rowst2 = (float2 *)(ws + a->rows * sizeof(float4) + 3 * pn * sizeof(float) + 256);   // (16-B aligned: rows % 32)
  // kl_dwo2_kernel's region (sized by cc_dec_kl_ws_size for rows > TR; 16-B aligned)
  p.dw_part = a->rows > TR ? (float *)(p.rowst2 + a->rows) : nullptr;
  hipStream_t s = as_stream(stream);
  const dim3 gs((unsigned)p.nsl), gm((unsigned)p.nsl);
  // many row tiles (full mode): dWo from the stored dZ by kl_dwo_kernel (even V: 4-B aligned rows);
  // one tile (the sampled regulariser): in the main pass, from its LDS dZ^T tile
  const bool dw_sep = a->rows > TR && a->V % 2 == 0;
  // the main pass's dZ through LDS as 16-B row stores (16-B aligned rows; the sentinel past range)
  const bool wstore = a->V % 8 == 0 && ((uintptr_t)a->dZ & 15) == 0 && (int64_t)a->rows * a->V * 2 < 0x80000000ll;
  // the stats in slice pairs x row halves (kl_stats2_kernel): many row tiles (full mode), d = 256
  const bool stats2 = CCREC_KL_STATS2 && a->d == 256 && a->rows > TR;
  // dWo in 192-column slices x two row halves (kl_dwo2_kernel): 16-B aligned rows, the chunk
  // sentinel 0x80000000 past dZ's range, at least one chunk per half
  const bool dwo2 = CCREC_DWO2 && a->d == 256 && a->V % 8 == 0 && (((uintptr_t)a->dZ | (uintptr_t)a->gW) & 15) == 0 &&
                    (int64_t)a->rows * a->V * 2 < 0x80000000ll && cdiv(a->rows, DW2_KC) >= DW2_SPLIT &&
                    p.dw_part && !(a->flags & CC_KL_DWO_NARROW);
#define KL_LAUNCH(DD)                                                                                          \
  if (a->d == DD) {                                                                                          \
    if (stats2 && DD == 256)                                                                                 \
      hipLaunchKernelGGL(kl_stats2_kernel, dim3((unsigned)cdiv(p.nsl, 2), 2), dim3(NTH), 0, s, p);          \
    else                                                                                                     \
      hipLaunchKernelGGL((kl_stats_kernel<DD>), gs, dim3(NTH), 0, s, p);                                    \
    CC_LAUNCH_CHECK("kl_stats_kernel");                                                                      \
    hipLaunchKernelGGL(kl_merge_kernel, dim3((unsigned)cdiv(a->rows, 4)), dim3(256), 0, s, p);              \
    CC_LAUNCH_CHECK("kl_merge_kernel");                                                                      \
    if (dw_sep) {                                                                                            \
      if (wstore)                                                                                            \
        hipLaunchKernelGGL((kl_main_kernel<DD, KL_SEP_CPOL, false, (DD <= 256)>), gm, dim3(NTH), 0, s, p);    \
      else                                                                                                   \
        hipLaunchKernelGGL((kl_main_kernel<DD, KL_SEP_CPOL, false>), gm, dim3(NTH), 0, s, p);                 \
      CC_LAUNCH_CHECK("kl_main_kernel");                                                                     \
      hipLaunchKernelGGL((kl_fix_kernel<DD, false>), dim3(FIXG), dim3(NTH), 0, s, p);                       \
      CC_LAUNCH_CHECK("kl_fix_kernel");                                                                      \
      const dim3 gd((unsigned)cdiv(a->V, DW_NB), (unsigned)(DD > 256 ? DD / 256 : 1));                     \
      if (dwo2 && DD == 256) {                                                                               \
        static const bool attr2 = hipFuncSetAttribute((const void *)kl_dwo2_kernel<256>,                     \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, DW2_LDS) == \
                                  hipSuccess;                                                                \
        CC_REQUIRE(attr2, "cc_dec_softmax_kl_dw: dynamic LDS attribute");                                    \
        hipLaunchKernelGGL((kl_dwo2_kernel<256>), dim3((unsigned)cdiv(a->V, DW2_NB), DW2_SPLIT), dim3(DW2_NT), \
                           DW2_LDS, s, p);                                                                   \
        CC_LAUNCH_CHECK("kl_dwo2_kernel");                                                                   \
        hipLaunchKernelGGL(kl_dwo2_sum_kernel, dim3(1024), dim3(256), 0, s, (const float4 *)p.dw_part,        \
                           (float4 *)p.gW, (int64_t)256 * a->V / 4);                                         \
      } else if (a->V % 8 == 0)                                                                              \
        hipLaunchKernelGGL((kl_dwo_kernel<DD, true>), gd, dim3(NTH), 0, s, p);                               \
      else                                                                                                   \
        hipLaunchKernelGGL((kl_dwo_kernel<DD, false>), gd, dim3(NTH), 0, s, p);                              \
      CC_LAUNCH_CHECK("kl_dwo_kernel");                                                                      \
    } else {                                                                                                 \
      if (a->rows > TR)                                                                                      \
        hipLaunchKernelGGL((kl_main_kernel<DD, KL_CPOL_NT, true>), gm, dim3(NTH), 0, s, p);                  \
      else                                                                                                   \
        hipLaunchKernelGGL((kl_main_kernel<DD, 0, true>), gm, dim3(NTH), 0, s, p);                           \
      CC_LAUNCH_CHECK("kl_main_kernel");                                                                     \
      hipLaunchKernelGGL((kl_fix_kernel<DD, true>), dim3(FIXG), dim3(NTH), 0, s, p);                        \
      CC_LAUNCH_CHECK("kl_fix_kernel");                                                                      \
    }                                                                                                        \
  }
  KL_LAUNCH(256)
  KL_LAUNCH(128)
  KL_LAUNCH(512)
#undef KL_LAUNCH
  return CC_OK;
}
