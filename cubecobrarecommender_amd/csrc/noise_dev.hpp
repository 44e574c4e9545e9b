// F's device code (noise.hip: the DAE input-noise function, generator.py:38-103) shared by the
// launches that host F's per-cube workgroups: cc_noise_fwd / the Adam + F launch (noise.hip) and
// the tower backward launch (tower.hip, cc_tower_bwd_chain_noise).  noise_block<NTT> runs one cube
// on NTT threads (any multiple of 64; a workgroup of k * NTT threads can run k cubes, each slice
// with its own LDS and s_k — every slice passes the same barriers); every draw is a pure function of
// (seed, step, slot, kind, index, try), so the result does not depend on NTT or on the launch.
#pragma once
#include "common.hpp"
#include "detmath.hpp"

// dev-only phase timestamps (tools/micro/noise_probe.hip defines it); compiled out of the library
#ifndef NOISE_PROBE
#define NOISE_PROBE(b, k)
#endif

namespace ccnoise {

#ifndef NOISE_NT
#define NOISE_NT 256
#endif
constexpr int NT = NOISE_NT;   // threads per cube (and per Adam block of the Adam + F launch)
static_assert(NT % 64 == 0 && NT <= 1024, "whole waves");
constexpr uint32_t KIND_NOISE = 0, KIND_CUT = 1, KIND_YCUT = 2, KIND_ADD = 3, KIND_ADD_FB = 4,
                   KIND_REG = 5;
constexpr int ADD_MAX_TRIES = 256;

__device__ __forceinline__ u32x4 rng(uint64_t seed, uint32_t step, uint32_t slot, uint32_t kind,
                                     uint32_t idx, uint32_t tries) {
  return philox4x32_10(idx, (kind << 24) | tries, slot, step, (uint32_t)seed,
                       (uint32_t)(seed >> 32));
}

// first index j with cdf[j] > u  (numpy searchsorted side='right').  With a guide table the answer
// lies in [guide[g], guide[g+1]], g = floor(u 2^G) (cdf is monotone and g/2^G <= u < (g+1)/2^G),
// and hi = min(guide[g+1], V-1) is itself a valid answer (cdf[guide[g+1]] > (g+1)/2^G > u, and
// cdf[V-1] = 1 > u), so the search runs over [lo, hi) with hi as the default: a bucket without a
// cdf boundary (guide[g] == guide[g+1], most of the 2^16) needs no cdf load at all, the others one
// dependent load fewer than a search over [lo, hi + 1).
__device__ __forceinline__ int search_right(const double *__restrict__ cdf, int V, double u,
                                            const int32_t *__restrict__ guide, int glog2) {
  int lo = 0, hi = V;
  if (guide) {
    const int g = (int)(u * (double)(1 << glog2));
    lo = guide[g];
    hi = min(guide[g + 1], V - 1);
  }
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] <= u)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < V ? lo : V - 1;
}

__device__ __forceinline__ double noise_level(double mean, double std, double z) {
#pragma clang fp contract(off)
  double lvl = mean + std * z;
  lvl = lvl < 0.05 ? 0.05 : lvl;
  return lvl > 0.8 ? 0.8 : lvl;
}

__device__ __forceinline__ bool bit_of(const uint32_t *bits, int j) {
  return (bits[j >> 5] >> (j & 31)) & 1u;
}

// Exact (rare) fallback: inverse CDF over the excludes by a sequential fp64 scan.
__device__ inline int add_fallback(const double *__restrict__ ns, int V, const uint32_t *cube_bits,
                            double u01) {
  double s = 0.0;
  for (int j = 0; j < V; ++j)
    if (!bit_of(cube_bits, j)) s += ns[j];
  if (!(s > 0.0)) return -1;
  const double u = u01 * s;
  double acc = 0.0;
  int last = -1;
  for (int j = 0; j < V; ++j) {
    if (bit_of(cube_bits, j)) continue;
    if (ns[j] > 0.0) last = j;
    acc += ns[j];
    if (acc > u) return j;
  }
  return last;
}

// F for cube slot b of the batch at (step, batch-in-epoch, epoch); smem: the dynamic LDS of
// cc_noise_fwd's launch.
template <int NTT = NT>
__device__ __forceinline__ void noise_block(const cc_noise_args &a, uint32_t *smem, int &s_k,
                                            int b, int64_t step64, int64_t batch, int64_t epoch) {
  const int VW = (a.V + 31) >> 5;
  uint32_t *cube_bits = smem;
  uint32_t *cut_bits = cube_bits + VW;
  uint32_t *ycut_bits = cut_bits + VW;
  uint32_t *add_bits = ycut_bits + VW;
  int32_t *scan = (int32_t *)(add_bits + VW);  // [NTT + 1]

  const int tid = threadIdx.x % NTT;   // (a workgroup of k * NTT threads runs k cubes, one per slice)
  const uint32_t slot = a.slot_base + (uint32_t)b;
  const uint32_t step = (uint32_t)step64;
  const int XW = (a.xt_rows + 31) >> 5;

  const int32_t *perm = a.perm + (epoch % a.num_perms) * (int64_t)a.num_cubes;
  const int32_t cube = perm[batch * (int64_t)a.batch_stride + a.batch_offset + b];
  const int64_t beg = a.cube_ptr[cube];
  const int n = (int)(a.cube_ptr[cube + 1] - beg);
  const int32_t *__restrict__ inc = a.cube_idx + beg;
  NOISE_PROBE(b, 0);

  for (int w = tid; w < 4 * VW; w += NTT) cube_bits[w] = 0u;
  __syncthreads();
  NOISE_PROBE(b, 1);
  for (int i = tid; i < n; i += NTT) {
    const int j = inc[i];
    atomicOr(&cube_bits[j >> 5], 1u << (j & 31));
  }
  if (tid == 0) {
    const u32x4 o = rng(a.seed, step, slot, KIND_NOISE, 0, 0);
    const double z = detm::det_normal(u53_open0(o.x, o.y), u53(o.z, o.w));
    const double lvl = noise_level(a.noise_mean, a.noise_std, z);
    int k = (int)((double)n * lvl);
    if (n + k > a.x_cap) {  // cannot happen when x_cap >= 1.8 * max cube size
      atomicOr(a.status, 1);
      k = a.x_cap - n > 0 ? a.x_cap - n : 0;
    }
    s_k = k;
  }
  __syncthreads();
  NOISE_PROBE(b, 2);
  const int k = s_k;
  // cut draws (with replacement from the includes)
  for (int i = tid; i < k; i += NTT) {
    const uint32_t pos = mulhi_bound(rng(a.seed, step, slot, KIND_CUT, (uint32_t)i, 0).x, (uint32_t)n);
    const int card = inc[pos];
    atomicOr(&cut_bits[card >> 5], 1u << (card & 31));
  }
  // ycut draws from the cut multiset: draw q picks cut draw qq, whose card is a pure function of
  // (qq, the cube) — recomputed here instead of read back from an LDS list, so the ycut draws need
  // no barrier after the cut draws
  const int nq = k >> 2;
  for (int q = tid; q < nq; q += NTT) {
    const uint32_t qq = mulhi_bound(rng(a.seed, step, slot, KIND_YCUT, (uint32_t)q, 0).x, (uint32_t)k);
    const uint32_t pos = mulhi_bound(rng(a.seed, step, slot, KIND_CUT, qq, 0).x, (uint32_t)n);
    const int card = inc[pos];
    atomicOr(&ycut_bits[card >> 5], 1u << (card & 31));
  }
  // add draws (rejection against the global CDF): they need only cube_bits, so they run beside the
  // cut and ycut draws
  for (int i = tid; i < k; i += NTT) {
    int pick = -1;
    for (int t = 0; t < ADD_MAX_TRIES; ++t) {
      const u32x4 o = rng(a.seed, step, slot, KIND_ADD, (uint32_t)i, (uint32_t)t);
      const int j = search_right(a.cdf, a.V, u53(o.x, o.y), a.guide, a.guide_log2);
      if (!bit_of(cube_bits, j)) {
        pick = j;
        break;
      }
    }
    if (pick < 0) {
      const u32x4 o = rng(a.seed, step, slot, KIND_ADD_FB, (uint32_t)i, 0);
      pick = add_fallback(a.neg_sampler, a.V, cube_bits, u53(o.x, o.y));
    }
    if (pick >= 0) atomicOr(&add_bits[pick >> 5], 1u << (pick & 31));
  }
  __syncthreads();
  NOISE_PROBE(b, 3);
  NOISE_PROBE(b, 4);
  // y bitmask: cube \ ycut (and x as a bitmask, for cc_embed_gather_fwd_xt's transpose)
  uint32_t *yrow = a.y_bits + (int64_t)b * VW;
  for (int w = tid; w < VW; w += NTT) yrow[w] = cube_bits[w] & ~ycut_bits[w];
  if (a.x_bits)
    for (int w = tid; w < VW; w += NTT)
      a.x_bits[(int64_t)b * VW + w] = (cube_bits[w] & ~cut_bits[w]) | add_bits[w];
  // x: sorted compaction of (cube \ cut) | add  — chunked block scan over the VW words
  const int per = (VW + NTT - 1) / NTT;
  const int w0 = tid * per, w1 = min(VW, w0 + per);
  int cnt = 0;
  for (int w = w0; w < w1; ++w) cnt += __popc((cube_bits[w] & ~cut_bits[w]) | add_bits[w]);
  // exclusive block scan of cnt: inclusive wave scan by shuffles, then the wave totals
  const int lane = tid & 63, wv = tid >> 6;
  int inc_sum = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc_sum, off);
    if (lane >= off) inc_sum += y;
  }
  if (lane == 63) scan[wv] = inc_sum;
  __syncthreads();
  NOISE_PROBE(b, 5);
  int wbase = 0;
#pragma unroll
  for (int w = 0; w < NTT / 64; ++w) wbase += w < wv ? scan[w] : 0;
  int total = 0;
#pragma unroll
  for (int w = 0; w < NTT / 64; ++w) total += scan[w];
  int pos = wbase + inc_sum - cnt;
  int32_t *xrow = a.x_idx + (int64_t)b * a.x_cap;
  for (int w = w0; w < w1; ++w) {
    uint32_t m = (cube_bits[w] & ~cut_bits[w]) | add_bits[w];
    while (m) {
      const int bit = __ffs(m) - 1;
      m &= m - 1;
      const int j = (w << 5) + bit;
      if (pos < a.x_cap) xrow[pos] = j;
      if (a.xt_bits) atomicOr(&a.xt_bits[(int64_t)j * XW + (b >> 5)], 1u << (b & 31));
      ++pos;
    }
  }
  if (tid == 0) a.x_cnt[b] = min(total, a.x_cap);
  NOISE_PROBE(b, 6);
  // regulariser row for this slot (generator.py:47-51): one draw ∝ neg_sampler
  if (a.with_reg && tid == 0) {
    const u32x4 o = rng(a.seed, step, slot, KIND_REG, 0, 0);
    const int j = search_right(a.cdf, a.V, u53(o.x, o.y), a.guide, a.guide_log2);
    a.reg_idx[b] = j;
    const int r = a.B + b;
    a.x_idx[(int64_t)r * a.x_cap] = j;
    a.x_cnt[r] = 1;
    // (xt_rows == B: the W1 gradient takes the reg rows by index, cc_embed_grad_cs_reg — no bit)
    if (a.xt_bits && r < a.xt_rows) atomicOr(&a.xt_bits[(int64_t)j * XW + (r >> 5)], 1u << (r & 31));
    s_k = j;
  }
  if (a.with_reg && a.x_bits) {  // the reg row {j} as a bitmask
    __syncthreads();
    const int j = s_k;
    uint32_t *xr = a.x_bits + (int64_t)(a.B + b) * VW;
    for (int w = tid; w < VW; w += NTT) xr[w] = w == (j >> 5) ? 1u << (j & 31) : 0u;
  }
}


}  // namespace ccnoise
