// cc_topn — ranking for the recommend path (src/scripts/ml_recommend.py:87-108,
// web/ml_recommend_web.py:46-64).
//
// The reference ranks with numpy `results.argsort()[::-1]` (default, unstable sort: its tie
// order is implementation-defined).  The pinned rule here is numpy argsort(kind='stable')[::-1]:
// descending probability, equal probabilities -> higher card index first.
//
// One 1024-thread workgroup: a stable LSD radix sort of the V fp32 probabilities (non-negative,
// so their bit patterns order like the values), 4 passes of 8 bits.  Each of the 16 waves owns a
// contiguous slice of the keys; per-digit ranks inside a wave come from a 64-lane ballot
// multisplit (8 ballots -> the set of lanes sharing my digit), so scatter order is stable.
// Keys/values ping-pong through a small global workspace (L2-resident).  Then additions = the
// first max(amount, 1) cards of the descending order that are not in the cube (block prefix scan),
// cut_vals[i] = probs[cube_idx[i]].
#include "common.hpp"

namespace {

constexpr int NT = 1024;
constexpr int NW = NT / 64;
constexpr int RADIX = 256;

__device__ __forceinline__ uint64_t match_digit(uint32_t dgt, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) {
    const bool b = (dgt >> bit) & 1u;
    const uint64_t bb = __ballot(b);
    m &= b ? bb : ~bb;
  }
  return m;
}

__device__ __forceinline__ int block_excl_scan(int v, int *sc, int *total) {
  // sc: [NT] scratch in LDS
  sc[threadIdx.x] = v;
  __syncthreads();
  for (int off = 1; off < NT; off <<= 1) {
    const int t = threadIdx.x >= off ? sc[threadIdx.x - off] : 0;
    __syncthreads();
    sc[threadIdx.x] += t;
    __syncthreads();
  }
  const int incl = sc[threadIdx.x];
  if (total) *total = sc[NT - 1];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(NT) void topn_kernel(const float *__restrict__ probs, int V,
                                                  const int32_t *__restrict__ cube_idx, int n,
                                                  int amount, int32_t *additions, int32_t *n_add,
                                                  float *add_vals, float *cut_vals,
                                                  int32_t *order_out, uint32_t *ws) {
  __shared__ uint32_t hist[RADIX * NW];  // [digit][wave]
  __shared__ int sc[NT];
  extern __shared__ __attribute__((aligned(16))) uint32_t cube_bits[];  // [ceil(V/32)]
  const int VW = (V + 31) >> 5;
  uint32_t *kA = ws, *kB = ws + V;
  int32_t *vA = (int32_t *)(ws + 2 * (int64_t)V), *vB = vA + V;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;

  for (int i = threadIdx.x; i < VW; i += NT) cube_bits[i] = 0u;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += NT) {
    const int j = cube_idx[i];
    atomicOr(&cube_bits[j >> 5], 1u << (j & 31));
    cut_vals[i] = probs[j];
  }

  const int S = (int)cdiv(cdiv(V, NW), 64) * 64;  // per-wave slice
  const int lo = w * S, hi = min(V, lo + S);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    const uint32_t *ksrc = (pass & 1) ? kB : kA;
    const int32_t *vsrc = (pass & 1) ? vB : vA;
    uint32_t *kdst = (pass & 1) ? kA : kB;
    int32_t *vdst = (pass & 1) ? vA : vB;
    for (int i = threadIdx.x; i < RADIX * NW; i += NT) hist[i] = 0u;
    __syncthreads();
    // histogram (per wave, per digit)
    for (int base = lo; base < hi; base += 64) {
      const int i = base + lane;
      const bool valid = i < hi;
      uint32_t key = 0;
      if (valid) key = pass == 0 ? __float_as_uint(probs[i]) : ksrc[i];
      const uint32_t dg = (key >> shift) & 0xFFu;
      const uint64_t m = match_digit(dg, valid);
      if (valid && (m & lt) == 0) hist[dg * NW + w] += (uint32_t)__popcll(m);
    }
    __syncthreads();
    // exclusive scan over [digit][wave]
    {
      constexpr int PER = RADIX * NW / NT;  // 4
      int loc[PER];
      int s = 0;
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        loc[e] = (int)hist[threadIdx.x * PER + e];
        s += loc[e];
      }
      int off = block_excl_scan(s, sc, nullptr);
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        hist[threadIdx.x * PER + e] = (uint32_t)off;
        off += loc[e];
      }
    }
    __syncthreads();
    // stable scatter
    for (int base = lo; base < hi; base += 64) {
      const int i = base + lane;
      const bool valid = i < hi;
      uint32_t key = 0;
      int32_t val = 0;
      if (valid) {
        key = pass == 0 ? __float_as_uint(probs[i]) : ksrc[i];
        val = pass == 0 ? i : vsrc[i];
      }
      const uint32_t dg = (key >> shift) & 0xFFu;
      const uint64_t m = match_digit(dg, valid);
      uint32_t basepos = 0;
      if (valid) basepos = hist[dg * NW + w];
      if (valid) {
        const uint32_t pos = basepos + (uint32_t)__popcll(m & lt);
        kdst[pos] = key;
        vdst[pos] = val;
      }
      if (valid && (m & lt) == 0) hist[dg * NW + w] = basepos + (uint32_t)__popcll(m);
    }
    __threadfence_block();
    __syncthreads();
  }
  // after 4 passes the ascending result is in kA/vA.  Descending position q <-> asc index V-1-q.
  const int want = amount > 0 ? amount : 1;
  int done = 0;
  for (int q0 = 0; q0 < V && done < want; q0 += NT) {
    const int q = q0 + threadIdx.x;
    int card = -1;
    bool ok = false;
    if (q < V) {
      card = vA[V - 1 - q];
      ok = !((cube_bits[card >> 5] >> (card & 31)) & 1u);
    }
    int total;
    const int pre = block_excl_scan(ok ? 1 : 0, sc, &total);
    if (ok && done + pre < want) {
      additions[done + pre] = card;
      add_vals[done + pre] = probs[card];
    }
    done += total;
  }
  if (order_out)
    for (int q = threadIdx.x; q < V; q += NT) order_out[q] = vA[V - 1 - q];
  if (threadIdx.x == 0) *n_add = done < want ? done : want;
}

}  // namespace

extern "C" size_t cc_topn_workspace_size(int32_t V) {
  return (size_t)4 * (4 * (size_t)V + 16);
}

extern "C" int cc_topn(const float *probs, int32_t V, const int32_t *cube_idx, int32_t n,
                       int32_t amount, int32_t *additions, int32_t *n_additions, float *add_vals,
                       float *cut_vals, int32_t *order, void *ws, void *stream) {
  CC_REQUIRE(probs && additions && n_additions && add_vals && ws, "cc_topn: null pointer");
  CC_REQUIRE(V > 0 && n >= 0 && n <= V, "cc_topn: bad V/n");
  CC_REQUIRE(n == 0 || (cube_idx && cut_vals), "cc_topn: cube_idx/cut_vals needed when n > 0");
  const size_t lds = (size_t)cdiv(V, 32) * 4;
  CC_REQUIRE(lds <= 96 * 1024, "cc_topn: V too large");
  hipLaunchKernelGGL(topn_kernel, dim3(1), dim3(NT), lds, as_stream(stream), probs, V, cube_idx, n,
                     amount, additions, n_additions, add_vals, cut_vals, order, (uint32_t *)ws);
  CC_LAUNCH_CHECK("topn_kernel");
  return CC_OK;
}
