// Card co-occurrence graph: SURVEY §8(f) row N1, the GPU create_adjacency_matrix.
//
// Reference: src/non_ml/utils.py:75-91 builds, card row by card row in numpy,
//   M[i, j] = |{cubes containing i and j}| / |{cubes containing i}|   (rows of unseen cards: 0)
// with an optional fill_diagonal(force_diag) (:90-91), and src/ml/train.py:69-71 turns it into
//   M~ = (M with diag := 1) / rowsum(M with diag := 1).
//
// Here the 0/1 cube matrix X [C, V] is held transposed as 4-bit FP4 (e2m1) codes, Xt [V][K]
// nibbles (1.0 = 0x2, K = cubes padded to 256), and counts = Xt Xt^T runs on the CDNA4
// block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4 with FP4 operands and unit E8M0 scales:
// 64 cubes per instruction at the cycles of a 32x32x16 bf16 one (4x the bf16 rate, half the
// bytes of int8), f32 accumulation exact for counts < 2^24 (chunks are capped below that).
// Only the upper triangle of 256x256 tiles is multiplied — counts is symmetric, so every tile
// stores itself and its mirror.  The normalisations fold into the epilogue with two per-card
// integers computed beforehand:
//   d_i = counts[i, i] = |{cubes containing i}|,
//   S_i = sum_j counts[i, j] = sum over cubes containing i of the cube's distinct size,
// so M[i, j] = counts/d_i (f64, the reference's dtype and file format, bit-exact: one correctly
// rounded division of exact integers) and M~[i, j] = counts/S_i (fp32, the dtype the D2 loss
// consumes; a row of an unseen card is e_i, as train.py:69-71 makes it).  Cubes may be
// processed in chunks (bounded Xt); partial counts then accumulate in an int32 [V][V] buffer.
#include <algorithm>

#include "common.hpp"

namespace {

typedef __attribute__((ext_vector_type(4))) int i32x4_t;
typedef __attribute__((ext_vector_type(8))) int i32x8_t;

constexpr int KPADC = 256;      // cube-axis padding of Xt rows (cubes) = 128 bytes of nibbles
constexpr int TB = 256;         // output tile edge (cards)
constexpr int BK = 128;         // bytes per row per stage (256 cubes)
constexpr int CH = BK / 16;     // 16-B chunks per LDS row
constexpr int NTH = 512;        // 8 waves: 2 (rows) x 4 (cols), each 128 x 64 outputs
constexpr int NL = TB * CH / NTH;  // 16-B loads per operand per thread per stage
constexpr int STAGE = TB * BK;  // bytes of one operand stage
constexpr int GS = 4;           // super-block edge (tiles): co-resident blocks share panels in L2
constexpr int EPR = 64;         // epilogue rows per LDS pass
constexpr int SP = TB + 1;      // epilogue LDS pitch (words)
constexpr uint32_t FP4_ONE = 0x2u;
constexpr int E8M0_ONE = 0x7f7f7f7f;  // scale 2^0 in every byte
constexpr int64_t MAX_CHUNK = (int64_t)1 << 24;  // f32 accumulators stay exact below 2^24

__host__ __device__ inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------ Xt build (one WG per cube)
// Xt nibble (j, c - c0) = FP4 1.0 for every card j of cube c (duplicates in a list collapse, as
// in the reference's dense cubes[c, ids] = 1, utils.py:72); ncnt[c - c0] = distinct size.
__global__ __launch_bounds__(256) void xt_scatter_kernel(const int32_t *__restrict__ row_ptr,
                                                        const int32_t *__restrict__ idx, int c0,
                                                        int V, int64_t Kb, uint8_t *xt,
                                                        int32_t *ncnt) {
  __shared__ int red[4];
  const int c = c0 + blockIdx.x;
  const int e0 = row_ptr[c], e1 = row_ptr[c + 1];
  const int64_t col = blockIdx.x;
  int first = 0;
  for (int e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    const int j = idx[e];
    if (j < 0 || j >= V) continue;  // the host wrapper validates ids; never write outside Xt
    const int64_t a = (int64_t)j * Kb + (col >> 1);
    uint32_t *w = reinterpret_cast<uint32_t *>(xt + (a & ~(int64_t)3));
    const uint32_t sh = 8u * (uint32_t)(a & 3) + 4u * (uint32_t)(col & 1);
    const uint32_t old = atomicOr(w, FP4_ONE << sh);
    first += ((old >> sh) & 0xfu) == 0u;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) first += __shfl_xor(first, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = first;
  __syncthreads();
  if (threadIdx.x == 0) ncnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------------ per-card d_i and S_i
// One WG per card row of Xt: d += set nibbles, S += the distinct sizes of those cubes.
__global__ __launch_bounds__(256) void card_stats_kernel(const uint8_t *__restrict__ xt,
                                                        int64_t Kb, int kc,
                                                        const int32_t *__restrict__ ncnt,
                                                        int64_t *d, int64_t *S) {
  __shared__ int64_t rd[4], rs[4];
  const int j = blockIdx.x;
  const uint4 *row = reinterpret_cast<const uint4 *>(xt + (int64_t)j * Kb);
  int64_t dd = 0, ss = 0;
  for (int q = threadIdx.x; q < (int)(Kb / 16); q += blockDim.x) {
    const uint4 v = row[q];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uint32_t x = w[t];
      while (x) {  // sparse: most rows are mostly zero
        const int nib = __builtin_ctz(x) >> 2;
        x &= ~(0xfu << (4 * nib));
        const int c = q * 32 + t * 8 + nib;
        if (c < kc) {
          dd += 1;
          ss += ncnt[c];
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    dd += __shfl_xor(dd, off);
    ss += __shfl_xor(ss, off);
  }
  if ((threadIdx.x & 63) == 0) {
    rd[threadIdx.x >> 6] = dd;
    rs[threadIdx.x >> 6] = ss;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    d[j] += rd[0] + rd[1] + rd[2] + rd[3];
    S[j] += rs[0] + rs[1] + rs[2] + rs[3];
  }
}

// ------------------------------------------------------------------ symmetric FP4 GEMM
struct CoParams {
  const uint8_t *xt;
  int64_t Kb;  // Xt row pitch in bytes (multiple of BK); the reduction runs over 2 * Kb cubes
  int V, nb, nsb;
  const int32_t *acc_in;  // partial counts of earlier cube chunks (or null)
  int32_t *counts;        // int32 [V][V] out (or null)
  double *adj;            // M  f64 [V][V] out (or null)
  float *adjn;            // M~ f32 [V][V] out (or null)
  const int64_t *d, *S;
  double force_diag;
  int has_force;
};

// Bijective: consecutive logical ids land on one XCD (blocks are dispatched round-robin).
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, x = b % 8, slot = b / 8;
  return x < r ? x * (q + 1) + slot : r * (q + 1) + (x - r) * q + slot;
}

// 16 bytes (32 FP4 codes) of row `row`, chunk c of a swizzled stage; the FP4 operand of the
// 32x32x64 MFMA occupies the low 4 registers (the backend allocates only those).
__device__ __forceinline__ i32x8_t co_frag(const uint8_t *S, int row, int c) {
  const i32x4_t v = *reinterpret_cast<const i32x4_t *>(S + row * BK + ((c ^ (row & (CH - 1))) * 16));
  return i32x8_t{v[0], v[1], v[2], v[3], 0, 0, 0, 0};
}

__device__ __forceinline__ double m_of(int32_t c, int64_t di, bool diag, const CoParams &p) {
  if (diag && p.has_force) return p.force_diag;
  return di != 0 ? (double)c / (double)di : (double)c;
}
__device__ __forceinline__ float mt_of(int32_t c, int64_t si, bool diag) {
  if (si == 0) return diag ? 1.f : 0.f;
  return (float)((double)c / (double)si);
}

// Write 4 consecutive outputs of row gi starting at column gj (row-major [V][V] targets).
__device__ __forceinline__ void co_store4(const CoParams &p, int gi, int gj, int32_t (&c)[4],
                                          int64_t di, int64_t si) {
  const int64_t o = (int64_t)gi * p.V + gj;
  const bool full = gj + 3 < p.V && (p.V & 3) == 0;
  if (p.acc_in) {
    if (full) {
      const int4 a = *reinterpret_cast<const int4 *>(p.acc_in + o);
      c[0] += a.x;
      c[1] += a.y;
      c[2] += a.z;
      c[3] += a.w;
    } else {
      for (int e = 0; e < 4 && gj + e < p.V; ++e) c[e] += p.acc_in[o + e];
    }
  }
  if (full) {
    if (p.counts) *reinterpret_cast<int4 *>(p.counts + o) = make_int4(c[0], c[1], c[2], c[3]);
    if (p.adj) {
      *reinterpret_cast<double2 *>(p.adj + o) =
          make_double2(m_of(c[0], di, gi == gj, p), m_of(c[1], di, gi == gj + 1, p));
      *reinterpret_cast<double2 *>(p.adj + o + 2) =
          make_double2(m_of(c[2], di, gi == gj + 2, p), m_of(c[3], di, gi == gj + 3, p));
    }
    if (p.adjn)
      *reinterpret_cast<float4 *>(p.adjn + o) =
          make_float4(mt_of(c[0], si, gi == gj), mt_of(c[1], si, gi == gj + 1),
                      mt_of(c[2], si, gi == gj + 2), mt_of(c[3], si, gi == gj + 3));
    return;
  }
  for (int e = 0; e < 4 && gj + e < p.V; ++e) {
    if (p.counts) p.counts[o + e] = c[e];
    if (p.adj) p.adj[o + e] = m_of(c[e], di, gi == gj + e, p);
    if (p.adjn) p.adjn[o + e] = mt_of(c[e], si, gi == gj + e);
  }
}

__global__ __launch_bounds__(NTH, 1) void cooccur_gemm_kernel(CoParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[4 * STAGE];
  __shared__ int64_t rowd[TB], rows_[TB], cold[TB], cols_[TB];

  // block -> (super-block pair, tile inside it); pairs (SI <= SJ) enumerated row by row
  const int64_t lid = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t sp = lid / (GS * GS);
  const int inner = (int)(lid % (GS * GS));
  int SI = 0;
  while (sp >= p.nsb - SI) {
    sp -= p.nsb - SI;
    ++SI;
  }
  const int SJ = SI + (int)sp;
  const int bi = SI * GS + inner / GS, bj = SJ * GS + inner % GS;
  if (bi >= p.nb || bj >= p.nb || bi > bj) return;  // whole block exits together
  const int bm = bi * TB, bn = bj * TB;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int wm = wave >> 2, wn = wave & 3;  // wave quadrant: rows wm*128.., cols wn*64..
  uint8_t *As = smem, *Bs = smem + 2 * STAGE;
  // staging plan: NL chunks of A and of B per thread (rows clamped: they feed discarded outputs)
  // (row indices, not 64-bit offsets: the loop is register-bound at 8 waves x 128 accumulators)
  int ga[NL], gb[NL], la[NL];
  const int ch16 = (threadIdx.x % CH) * 16;  // NTH % CH == 0: the same chunk for every i
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int v = threadIdx.x + NTH * i, row = v / CH, ch = v % CH;
    ga[i] = min(bm + row, p.V - 1);
    gb[i] = min(bn + row, p.V - 1);
    la[i] = row * BK + ((ch ^ (row & (CH - 1))) * 16);
  }
  const uint8_t *xtc = p.xt + ch16;
  f32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (int)(p.Kb / BK);
  i32x4_t ra[NL], rb[NL];
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      ra[i] = *reinterpret_cast<const i32x4_t *>(xtc + (int64_t)ga[i] * p.Kb);
      rb[i] = *reinterpret_cast<const i32x4_t *>(xtc + (int64_t)gb[i] * p.Kb);
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      *reinterpret_cast<i32x4_t *>(As + la[i]) = ra[i];
      *reinterpret_cast<i32x4_t *>(Bs + la[i]) = rb[i];
    }
  }
  __syncthreads();
  const int ar = wm * 128 + (lane & 31), br = wn * 64 + (lane & 31);
  for (int t = 0; t < nk; ++t) {
    // next stage in flight during this stage's MFMAs (the last iteration reloads its own
    // stage into the idle buffer: unconditional loads keep the ring in registers)
    const int64_t kn = (int64_t)min(t + 1, nk - 1) * BK;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      ra[i] = *reinterpret_cast<const i32x4_t *>(xtc + (int64_t)ga[i] * p.Kb + kn);
      rb[i] = *reinterpret_cast<const i32x4_t *>(xtc + (int64_t)gb[i] * p.Kb + kn);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs (hipcc sinks them)
    const uint8_t *as = As + (t & 1) * STAGE, *bs = Bs + (t & 1) * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int c = 2 * kk + half;  // lane half h holds cubes 64kk + 32h + (0..31), A and B alike
      i32x8_t a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = co_frag(as, ar + 32 * i, c);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = co_frag(bs, br + 32 * j, c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              a[i], b[j], acc[i][j], 4, 4, 0, E8M0_ONE, 0, E8M0_ONE);
    }
    uint8_t *na = As + ((t + 1) & 1) * STAGE, *nbp = Bs + ((t + 1) & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      *reinterpret_cast<i32x4_t *>(na + la[i]) = ra[i];
      *reinterpret_cast<i32x4_t *>(nbp + la[i]) = rb[i];
    }
    __syncthreads();
  }

  // ---- epilogue: counts tile -> LDS (passes of EPR rows) -> rows of the tile and its mirror
  if (threadIdx.x < TB) {
    const int r = threadIdx.x;
    rowd[r] = bm + r < p.V ? p.d[bm + r] : 0;
    rows_[r] = bm + r < p.V ? p.S[bm + r] : 0;
    cold[r] = bn + r < p.V ? p.d[bn + r] : 0;
    cols_[r] = bn + r < p.V ? p.S[bn + r] : 0;
  }
  float *T = reinterpret_cast<float *>(smem);  // [EPR][SP]
#pragma unroll
  for (int ps = 0; ps < TB / EPR; ++ps) {
    const int r0 = ps * EPR;
    __syncthreads();  // previous pass's readers are done (first pass: rowd/cold published)
    if (wm == (ps >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * (ps & 1) + ii;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int lc = wn * 64 + j * 32 + (lane & 31);
          const int lr0 = wm * 128 + i * 32 + 4 * half - r0;
#pragma unroll
          for (int r = 0; r < 16; ++r) T[(lr0 + (r & 3) + 8 * (r >> 2)) * SP + lc] = acc[i][j][r];
        }
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < EPR * (TB / 4); q += NTH) {
      const int lr = q / (TB / 4), lc = (q % (TB / 4)) * 4;
      const int gi = bm + r0 + lr, gj = bn + lc;
      if (gi >= p.V || gj >= p.V) continue;
      int32_t c[4] = {(int32_t)T[lr * SP + lc], (int32_t)T[lr * SP + lc + 1],
                      (int32_t)T[lr * SP + lc + 2], (int32_t)T[lr * SP + lc + 3]};
      co_store4(p, gi, gj, c, rowd[r0 + lr], rows_[r0 + lr]);
    }
    if (bi != bj) {  // mirror: rows bn + lc of the output, columns bm + r0 + lr .. +3
      for (int q = threadIdx.x; q < TB * (EPR / 4); q += NTH) {
        const int lc = q / (EPR / 4), lr = (q % (EPR / 4)) * 4;
        const int gi = bn + lc, gj = bm + r0 + lr;
        if (gi >= p.V || gj >= p.V) continue;
        int32_t c[4] = {(int32_t)T[lr * SP + lc], (int32_t)T[(lr + 1) * SP + lc],
                        (int32_t)T[(lr + 2) * SP + lc], (int32_t)T[(lr + 3) * SP + lc]};
        co_store4(p, gi, gj, c, cold[lc], cols_[lc]);
      }
    }
  }
}

struct CoWs {
  uint8_t *xt;
  int32_t *ncnt, *acc;
  int64_t *d, *S;
};
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
inline int64_t chunk_cubes_of(int32_t C, int32_t chunk) {
  int64_t kc = chunk > 0 && chunk < C ? chunk : C;
  return std::min<int64_t>(kc, MAX_CHUNK);
}
inline int64_t chunk_bytes(int32_t C, int32_t chunk) {  // Xt row pitch
  return cdiv64(chunk_cubes_of(C, chunk), KPADC) * KPADC / 2;
}
inline size_t ws_fixed_bytes(int32_t V, int32_t C, int32_t chunk) {
  const int64_t Kb = chunk_bytes(C, chunk), kc = chunk_cubes_of(C, chunk);
  return al256((size_t)V * Kb) + al256((size_t)(kc + 1) * 4) + 2 * al256((size_t)V * 8);
}
inline CoWs co_ws_of(void *base, int32_t V, int32_t C, int32_t chunk) {
  const int64_t Kb = chunk_bytes(C, chunk), kc = chunk_cubes_of(C, chunk);
  char *p = reinterpret_cast<char *>(base);
  CoWs w;
  w.xt = reinterpret_cast<uint8_t *>(p);
  p += al256((size_t)V * Kb);
  w.ncnt = reinterpret_cast<int32_t *>(p);
  p += al256((size_t)(kc + 1) * 4);
  w.d = reinterpret_cast<int64_t *>(p);
  p += al256((size_t)V * 8);
  w.S = reinterpret_cast<int64_t *>(p);
  p += al256((size_t)V * 8);
  w.acc = reinterpret_cast<int32_t *>(p);
  return w;
}
inline int n_chunks(int32_t C, int32_t chunk) {
  const int64_t kc = chunk_cubes_of(C, chunk);
  return C > 0 ? (int)cdiv64(C, kc) : 1;
}

}  // namespace

extern "C" {

size_t cc_adjacency_ws_size(int32_t V, int32_t C, int32_t chunk_cubes, int32_t with_counts) {
  if (V <= 0 || C < 0) return 0;
  size_t b = ws_fixed_bytes(V, C, chunk_cubes);
  // acc (int32 [V][V]) only when cubes come in several chunks and counts is not an output
  // (counts then doubles as the accumulator)
  if (n_chunks(C, chunk_cubes) > 1 && !with_counts) b += al256((size_t)V * V * 4);
  return b + 256;
}

int cc_adjacency(const int32_t *row_ptr, const int32_t *idx, int32_t C, int32_t V,
                 int32_t chunk_cubes, const double *force_diag, void *ws, int32_t *counts,
                 double *adj, float *adj_norm, void *stream) {
  CC_REQUIRE(V > 0 && C >= 0, "cc_adjacency: V > 0 and C >= 0 required");
  CC_REQUIRE(ws != nullptr, "cc_adjacency: workspace required");
  CC_REQUIRE(C == 0 || (row_ptr != nullptr && idx != nullptr), "cc_adjacency: null lists");
  CC_REQUIRE(counts || adj || adj_norm, "cc_adjacency: no output requested");
  CC_REQUIRE((int64_t)V * V < ((int64_t)1 << 40), "cc_adjacency: V too large");
  hipStream_t s = as_stream(stream);
  const int64_t kc = chunk_cubes_of(C, chunk_cubes);
  const int nchunks = n_chunks(C, chunk_cubes);
  CoWs w = co_ws_of(ws, V, C, chunk_cubes);
  int32_t *acc = nchunks > 1 ? (counts ? counts : w.acc) : nullptr;
  CC_HIP(hipMemsetAsync(w.d, 0, (size_t)V * 8, s));
  CC_HIP(hipMemsetAsync(w.S, 0, (size_t)V * 8, s));

  CoParams p{};
  p.V = V;
  p.nb = (int)cdiv64(V, TB);
  p.nsb = (int)cdiv64(p.nb, GS);
  p.d = w.d;
  p.S = w.S;
  p.has_force = force_diag != nullptr;
  p.force_diag = force_diag ? *force_diag : 0.0;
  const int64_t pairs = (int64_t)p.nsb * (p.nsb + 1) / 2;
  const int64_t blocks = pairs * GS * GS;
  CC_REQUIRE(blocks < ((int64_t)1 << 31), "cc_adjacency: V too large for one launch");

  for (int ch = 0; ch < nchunks; ++ch) {
    const int c0 = (int)(ch * kc);
    const int nc = C > 0 ? (int)std::min<int64_t>(kc, (int64_t)C - c0) : 0;
    const int64_t Kb = nc > 0 ? cdiv64(nc, KPADC) * KPADC / 2 : 0;
    if (nc > 0) {
      CC_HIP(hipMemsetAsync(w.xt, 0, (size_t)V * Kb, s));
      hipLaunchKernelGGL(xt_scatter_kernel, dim3(nc), dim3(256), 0, s, row_ptr, idx, c0, V, Kb,
                         w.xt, w.ncnt);
      CC_LAUNCH_CHECK("xt_scatter_kernel");
      hipLaunchKernelGGL(card_stats_kernel, dim3(V), dim3(256), 0, s, w.xt, Kb, nc, w.ncnt, w.d,
                         w.S);
      CC_LAUNCH_CHECK("card_stats_kernel");
    }
    const bool last = ch == nchunks - 1;
    p.xt = w.xt;
    p.Kb = Kb;
    p.acc_in = ch > 0 ? acc : nullptr;
    p.counts = last ? counts : acc;
    p.adj = last ? adj : nullptr;
    p.adjn = last ? adj_norm : nullptr;
    hipLaunchKernelGGL(cooccur_gemm_kernel, dim3((unsigned)blocks), dim3(NTH), 0, s, p);
    CC_LAUNCH_CHECK("cooccur_gemm_kernel");
  }
  return CC_OK;
}

}  // extern "C"
