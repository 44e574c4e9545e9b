// Card co-occurrence graph: SURVEY §8(f) row N1, the GPU create_adjacency_matrix.
//
// Reference: src/non_ml/utils.py:75-91 builds, card row by card row in numpy,
//   M[i, j] = |{cubes containing i and j}| / |{cubes containing i}|   (rows of unseen cards: 0)
// with an optional fill_diagonal(force_diag) (:90-91), and src/ml/train.py:69-71 turns it into
//   M~ = (M with diag := 1) / rowsum(M with diag := 1).
//
// Here the 0/1 cube matrix X [C, V] is held transposed, Xt [V][K] bytes (K = cubes padded to
// 128), and counts = Xt Xt^T is an int8 MFMA GEMM (v_mfma_i32_32x32x32_i8: exact int32
// counts, twice the bf16 rate) over the upper triangle of 128x128 tiles only — counts is
// symmetric, so every tile stores itself and its mirror.  The normalisations fold into the
// epilogue with two per-card integers computed beforehand:
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
typedef __attribute__((ext_vector_type(16))) int i32x16_t;

constexpr int KPAD = 128;   // cube-axis padding of Xt rows (bytes)
constexpr int TB = 128;     // output tile edge
constexpr int BK = 128;     // K bytes per stage
constexpr int CH = BK / 16; // 16-B chunks per LDS row
constexpr int NTH = 256;    // 4 waves, each a 64x64 quadrant
constexpr int NA = TB * CH / NTH;
constexpr int GS = 8;       // super-block edge (tiles): a launch's neighbours share panels in L2
constexpr int SP = TB + 1;  // epilogue LDS pitch (words)

__host__ __device__ inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------ Xt build (one WG per cube)
// Xt[j][c - c0] = 1 for every card j of cube c (duplicates in a list collapse, as in the
// reference's dense cubes[c, ids] = 1, utils.py:72); ncnt[c - c0] = the cube's distinct size.
__global__ __launch_bounds__(256) void xt_scatter_kernel(const int32_t *__restrict__ row_ptr,
                                                        const int32_t *__restrict__ idx, int c0,
                                                        int V, int64_t K, uint8_t *xt,
                                                        int32_t *ncnt) {
  __shared__ int red[4];
  const int c = c0 + blockIdx.x;
  const int e0 = row_ptr[c], e1 = row_ptr[c + 1];
  const int64_t col = blockIdx.x;
  int first = 0;
  for (int e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    const int j = idx[e];
    if (j < 0 || j >= V) continue;  // the host wrapper validates ids; never write outside Xt
    const int64_t a = (int64_t)j * K + col;
    uint32_t *w = reinterpret_cast<uint32_t *>(xt + (a & ~(int64_t)3));
    const uint32_t sh = 8u * (uint32_t)(a & 3);
    const uint32_t old = atomicOr(w, 1u << sh);
    first += ((old >> sh) & 0xffu) == 0u;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) first += __shfl_xor(first, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = first;
  __syncthreads();
  if (threadIdx.x == 0) ncnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------------ per-card d_i and S_i
// One WG per card row of Xt: d += popcount, S += sum of the distinct sizes of its cubes.
__global__ __launch_bounds__(256) void card_stats_kernel(const uint8_t *__restrict__ xt,
                                                        int64_t K, int kc,
                                                        const int32_t *__restrict__ ncnt,
                                                        int64_t *d, int64_t *S) {
  __shared__ int64_t rd[4], rs[4];
  const int j = blockIdx.x;
  const uint4 *row = reinterpret_cast<const uint4 *>(xt + (int64_t)j * K);
  int64_t dd = 0, ss = 0;
  for (int q = threadIdx.x; q < (int)(K / 16); q += blockDim.x) {
    const uint4 v = row[q];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uint32_t x = w[t];
      while (x) {  // sparse: most rows are mostly zero
        const int b = __builtin_ctz(x) >> 3;
        x &= ~(0xffu << (8 * b));
        const int c = q * 16 + t * 4 + b;
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

// ------------------------------------------------------------------ symmetric int8 GEMM
struct CoParams {
  const uint8_t *xt;
  int64_t K;  // Xt row pitch = reduction length (bytes, multiple of KPAD)
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

__device__ __forceinline__ i32x4_t co_frag(const uint8_t *S, int row, int c) {
  return *reinterpret_cast<const i32x4_t *>(S + row * BK + ((c ^ (row & (CH - 1))) * 16));
}

// Output value of count c at (i, j); ROWS: per-tile d/S of row i.
struct CoOut {
  __device__ __forceinline__ static double m_of(int32_t c, int64_t di, bool diag,
                                                const CoParams &p) {
    if (diag && p.has_force) return p.force_diag;
    return di != 0 ? (double)c / (double)di : (double)c;
  }
  __device__ __forceinline__ static float mt_of(int32_t c, int64_t si, bool diag) {
    if (si == 0) return diag ? 1.f : 0.f;
    return (float)((double)c / (double)si);
  }
};

// Write 4 consecutive outputs of row gi starting at column gj (row-major [V][V] targets).
__device__ __forceinline__ void co_store4(const CoParams &p, int gi, int gj, int32_t c[4],
                                          int64_t di, int64_t si) {
  const int64_t o = (int64_t)gi * p.V + gj;
  const bool full = gj + 3 < p.V && (p.V & 3) == 0;
  if (p.acc_in) {
    if (full) {
      const int4 a = *reinterpret_cast<const int4 *>(p.acc_in + o);
      c[0] += a.x; c[1] += a.y; c[2] += a.z; c[3] += a.w;
    } else {
      for (int e = 0; e < 4 && gj + e < p.V; ++e) c[e] += p.acc_in[o + e];
    }
  }
  if (full) {
    if (p.counts) *reinterpret_cast<int4 *>(p.counts + o) = make_int4(c[0], c[1], c[2], c[3]);
    if (p.adj) {
      double m[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = CoOut::m_of(c[e], di, gi == gj + e, p);
      *reinterpret_cast<double2 *>(p.adj + o) = make_double2(m[0], m[1]);
      *reinterpret_cast<double2 *>(p.adj + o + 2) = make_double2(m[2], m[3]);
    }
    if (p.adjn) {
      float m[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = CoOut::mt_of(c[e], si, gi == gj + e);
      *reinterpret_cast<float4 *>(p.adjn + o) = make_float4(m[0], m[1], m[2], m[3]);
    }
    return;
  }
  for (int e = 0; e < 4 && gj + e < p.V; ++e) {
    if (p.counts) p.counts[o + e] = c[e];
    if (p.adj) p.adj[o + e] = CoOut::m_of(c[e], di, gi == gj + e, p);
    if (p.adjn) p.adjn[o + e] = CoOut::mt_of(c[e], si, gi == gj + e);
  }
}

__global__ __launch_bounds__(NTH) void cooccur_gemm_kernel(CoParams p) {
  constexpr int STAGE = TB * BK;  // bytes of one A (or B) stage; A and B are double-buffered
  constexpr int LDS = 4 * STAGE > TB * SP * 4 ? 4 * STAGE : TB * SP * 4;
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS];
  __shared__ int64_t rowd[TB], rows_[TB], cold[TB], cols_[TB];

  // block -> (super-block pair, tile inside it); pairs (SI <= SJ) enumerated row by row
  const int64_t nblk = (int64_t)gridDim.x;
  const int64_t lid = xcd_remap(blockIdx.x, nblk);
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
  const int wm = wave >> 1, wn = wave & 1;
  uint8_t *As = smem, *Bs = smem + 2 * STAGE;
  // staging plan: NA chunks of A and of B per thread (rows clamped: they feed discarded outputs)
  int64_t ga[NA], gb[NA];
  int la[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int v = threadIdx.x + NTH * i, row = v / CH, ch = v % CH;
    ga[i] = (int64_t)min(bm + row, p.V - 1) * p.K + ch * 16;
    gb[i] = (int64_t)min(bn + row, p.V - 1) * p.K + ch * 16;
    la[i] = row * BK + ((ch ^ (row & (CH - 1))) * 16);
  }
  i32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  const int nk = (int)(p.K / BK);
  uint4 ra[NA], rb[NA];
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      ra[i] = *reinterpret_cast<const uint4 *>(p.xt + ga[i]);
      rb[i] = *reinterpret_cast<const uint4 *>(p.xt + gb[i]);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      *reinterpret_cast<uint4 *>(As + la[i]) = ra[i];
      *reinterpret_cast<uint4 *>(Bs + la[i]) = rb[i];
    }
  }
  __syncthreads();
  const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31);
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) {  // next stage in flight during this stage's MFMAs
      const int64_t k0 = (int64_t)(t + 1) * BK;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        ra[i] = *reinterpret_cast<const uint4 *>(p.xt + ga[i] + k0);
        rb[i] = *reinterpret_cast<const uint4 *>(p.xt + gb[i] + k0);
      }
    }
    const uint8_t *as = As + (t & 1) * STAGE, *bs = Bs + (t & 1) * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int c = 2 * kk + half;  // lane half h holds k = 32kk + 16h + j (same for A and B)
      const i32x4_t a0 = co_frag(as, ar, c), a1 = co_frag(as, ar + 32, c);
      const i32x4_t b0 = co_frag(bs, br, c), b1 = co_frag(bs, br + 32, c);
      acc[0][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (t + 1 < nk) {
      uint8_t *na = As + ((t + 1) & 1) * STAGE, *nbp = Bs + ((t + 1) & 1) * STAGE;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        *reinterpret_cast<uint4 *>(na + la[i]) = ra[i];
        *reinterpret_cast<uint4 *>(nbp + la[i]) = rb[i];
      }
    }
    __syncthreads();
  }

  // ---- epilogue: counts tile -> LDS -> coalesced rows of the tile and of its mirror
  if (threadIdx.x < TB) {
    const int r = threadIdx.x;
    rowd[r] = bm + r < p.V ? p.d[bm + r] : 0;
    rows_[r] = bm + r < p.V ? p.S[bm + r] : 0;
    cold[r] = bn + r < p.V ? p.d[bn + r] : 0;
    cols_[r] = bn + r < p.V ? p.S[bn + r] : 0;
  }
  int32_t *T = reinterpret_cast<int32_t *>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lc = wn * 64 + j * 32 + (lane & 31);
      const int lr0 = wm * 64 + i * 32 + 4 * half;
#pragma unroll
      for (int r = 0; r < 16; ++r) T[(lr0 + (r & 3) + 8 * (r >> 2)) * SP + lc] = acc[i][j][r];
    }
  __syncthreads();
  for (int q = threadIdx.x; q < TB * (TB / 4); q += NTH) {
    const int lr = q / (TB / 4), lc = (q % (TB / 4)) * 4;
    const int gi = bm + lr, gj = bn + lc;
    if (gi >= p.V || gj >= p.V) continue;
    int32_t c[4] = {T[lr * SP + lc], T[lr * SP + lc + 1], T[lr * SP + lc + 2], T[lr * SP + lc + 3]};
    co_store4(p, gi, gj, c, rowd[lr], rows_[lr]);
  }
  if (bi != bj) {  // mirror: row bn + lc of the output, columns bm + lr .. +3
    for (int q = threadIdx.x; q < TB * (TB / 4); q += NTH) {
      const int lc = q / (TB / 4), lr = (q % (TB / 4)) * 4;
      const int gi = bn + lc, gj = bm + lr;
      if (gi >= p.V || gj >= p.V) continue;
      int32_t c[4] = {T[lr * SP + lc], T[(lr + 1) * SP + lc], T[(lr + 2) * SP + lc],
                      T[(lr + 3) * SP + lc]};
      co_store4(p, gi, gj, c, cold[lc], cols_[lc]);
    }
  }
}

struct CoWs {
  uint8_t *xt;
  int32_t *ncnt, *acc;
  int64_t *d, *S;
};
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
inline int64_t chunk_k(int32_t C, int32_t chunk) {
  const int64_t kc = chunk > 0 && chunk < C ? chunk : C;
  return cdiv64(kc, KPAD) * KPAD;
}
// acc (int32 [V][V]) is only needed when cubes come in several chunks and no counts output
// is requested (otherwise counts doubles as the accumulator).
inline size_t co_ws_bytes(int32_t V, int32_t C, int32_t chunk, bool need_acc) {
  const int64_t K = chunk_k(C, chunk);
  size_t b = al256((size_t)V * K) + al256((size_t)K * 4) + 2 * al256((size_t)V * 8);
  if (need_acc) b += al256((size_t)V * V * 4);
  return b + 256;
}
inline CoWs co_ws_of(void *base, int32_t V, int32_t C, int32_t chunk) {
  const int64_t K = chunk_k(C, chunk);
  char *p = reinterpret_cast<char *>(base);
  CoWs w;
  w.xt = reinterpret_cast<uint8_t *>(p);
  p += al256((size_t)V * K);
  w.ncnt = reinterpret_cast<int32_t *>(p);
  p += al256((size_t)K * 4);
  w.d = reinterpret_cast<int64_t *>(p);
  p += al256((size_t)V * 8);
  w.S = reinterpret_cast<int64_t *>(p);
  p += al256((size_t)V * 8);
  w.acc = reinterpret_cast<int32_t *>(p);
  return w;
}

}  // namespace

extern "C" {

size_t cc_adjacency_ws_size(int32_t V, int32_t C, int32_t chunk_cubes, int32_t with_counts) {
  if (V <= 0 || C < 0) return 0;
  const int64_t kc = chunk_k(C, chunk_cubes);
  const bool multi = kc > 0 && cdiv64(C, kc) > 1;
  return co_ws_bytes(V, C, chunk_cubes, multi && !with_counts);
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
  const int64_t K = chunk_k(C, chunk_cubes);
  const int64_t kc_cubes = chunk_cubes > 0 && chunk_cubes < C ? chunk_cubes : C;
  const int nchunks = C > 0 ? (int)cdiv64(C, kc_cubes) : 1;
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
    const int c0 = (int)(ch * kc_cubes);
    const int nc = C > 0 ? (int)std::min<int64_t>(kc_cubes, C - c0) : 0;
    const int64_t Kch = nc > 0 ? cdiv64(nc, KPAD) * KPAD : 0;
    if (nc > 0) {
      CC_HIP(hipMemsetAsync(w.xt, 0, (size_t)V * Kch, s));
      hipLaunchKernelGGL(xt_scatter_kernel, dim3(nc), dim3(256), 0, s, row_ptr, idx, c0, V, Kch,
                         w.xt, w.ncnt);
      CC_LAUNCH_CHECK("xt_scatter_kernel");
      hipLaunchKernelGGL(card_stats_kernel, dim3(V), dim3(256), 0, s, w.xt, Kch, nc, w.ncnt, w.d,
                         w.S);
      CC_LAUNCH_CHECK("card_stats_kernel");
    }
    const bool last = ch == nchunks - 1;
    p.xt = w.xt;
    p.K = Kch;
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
