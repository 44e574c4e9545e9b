// cc_topn — ranking for the recommend path (src/scripts/ml_recommend.py:87-108,
// web/ml_recommend_web.py:46-64).
//
// The reference ranks with numpy `results.argsort()[::-1]` (default, unstable sort: its tie
// order is implementation-defined).  The pinned rule here is numpy argsort(kind='stable')[::-1]:
// descending probability, equal probabilities -> higher card index first.
//
// Additions (the request path): a stable LSD radix sort of the V cards spread over ceil(V/1024)
// workgroups ("tiles" of 1024 positions), 4 passes of 8 bits over the key
//     key'(card) = in_cube ? 0 : float_bits(prob) + 1          (probabilities are in [0, 1])
// so cube cards sink below every candidate and the additions are simply the first
// min(max(amount,1), V - n) cards of the descending order — no compaction pass.
//   topn_init_kernel: keys/ids of tile t, cut values, pass-0 digit histogram of the tile.
//   topn_pass_kernel: every tile reads all tiles' histograms for its digit bases, ranks its
//     items stably (per wave: 64-lane ballot multisplit; across waves: per-wave digit counts),
//     scatters them, and counts the NEXT pass's digits per destination tile with global
//     atomics (counts only, so the result does not depend on atomic order).  The last pass
//     writes the additions directly.
// Six launches, all tiles in parallel; nothing here depends on scheduling order.
//
// Full ranking (`order` != NULL; tests and tools): one 1024-thread workgroup runs the same
// stable sort with keys/ids ping-ponging through the global workspace (topn_full_kernel).
#include "common.hpp"
#include "topn_tiles.hpp"

namespace {

constexpr int FNT = 1024;  // full-ranking workgroup
constexpr int FNW = FNT / 64;
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

// Exclusive scan over the block of one int per thread; wtot: [blockDim/64] LDS scratch.
template <int THREADS>
__device__ __forceinline__ int block_excl_scan2(int v, int *wtot, int *total) {
  constexpr int W = THREADS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  int before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const int t = wtot[i];
    before += i < w ? t : 0;
    all += t;
  }
  __syncthreads();
  if (total) *total = all;
  return before + x - v;
}

// ------------------------------------------------------------------ tiled request path
template <int BITS>
__device__ __forceinline__ uint64_t match_bits(uint32_t dgt, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int bit = 0; bit < BITS; ++bit) {
    const bool b = (dgt >> bit) & 1u;
    const uint64_t bb = __ballot(b);
    m &= b ? bb : ~bb;
  }
  return m;
}

// cc_topn entry: keys/ids of tile t, its pass-0 histogram; H[1..] zeroed.
__global__ __launch_bounds__(tiles::NT) void topn_init_kernel(const float *__restrict__ probs,
                                                              int V, const int32_t *__restrict__ cube_idx,
                                                              int n, tiles::Ws w, int ntiles) {
  using namespace tiles;
  __shared__ uint32_t bits[TILE / 32];
  __shared__ uint32_t hist[R];
  const int t = blockIdx.x;
  const int lo = t * TILE;
  if (threadIdx.x < TILE / 32) bits[threadIdx.x] = 0u;
  for (int i = threadIdx.x; i < R; i += NT) hist[i] = 0u;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += NT) {
    const int j = cube_idx[i];
    if (j >= lo && j < lo + TILE) atomicOr(&bits[(j - lo) >> 5], 1u << ((j - lo) & 31));
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int pos = lo + it * NT + threadIdx.x;
    if (pos < V) {
      const int o = pos - lo;
      const uint32_t key = key_of(probs[pos], (bits[o >> 5] >> (o & 31)) & 1u);
      w.kA[pos] = key;
      w.iA[pos] = (uint32_t)pos;
      atomicAdd(&hist[digit(key, 0)], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += NT) {
    w.H[(int64_t)t * R + i] = hist[i];
#pragma unroll
    for (int p = 1; p < PASSES; ++p) w.H[((int64_t)p * ntiles + t) * R + i] = 0u;
  }
}

// One LSD pass over all tiles.  Tile t: stable ranks of its 1024 items (wave: ballot multisplit;
// across its 4 waves: per-wave digit counts), digit bases from every tile's histogram, scatter,
// and the next pass's [dest tile][digit] counts (aggregated in LDS, flushed with atomics).
__global__ __launch_bounds__(tiles::NT) void topn_pass_kernel(int pass, int V, int ntiles,
                                                              tiles::Ws w, const float *probs,
                                                              tiles::Req rq, tiles::Outs o) {
  using namespace tiles;
  extern __shared__ __attribute__((aligned(16))) uint32_t hs[];  // [min(tiles,32)][R]
  __shared__ uint32_t gbase[R];
  __shared__ uint32_t wcnt[NT / 64][R];
  __shared__ int wtot[NT / 64];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const bool last = pass == PASSES - 1;
  const bool local = ntiles <= LOCAL_TILES;
  const uint32_t *ksrc = (pass & 1) ? w.kB : w.kA, *isrc = (pass & 1) ? w.iB : w.iA;
  uint32_t *kdst = (pass & 1) ? w.kA : w.kB, *idst = (pass & 1) ? w.iA : w.iB;
  const uint32_t *Hp = w.H + (int64_t)pass * ntiles * R;

  // wave wv owns tile positions [wv*256, wv*256+256), 64 at a time (stable order = position)
  uint32_t key[IT], id[IT], rk[IT];
  const int base = t * TILE + wv * 256 + lane;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int pos = base + it * 64;
    key[it] = pos < V ? ksrc[pos] : 0u;
    id[it] = pos < V ? isrc[pos] : 0u;
  }
  for (int i = threadIdx.x; i < (NT / 64) * R; i += NT) (&wcnt[0][0])[i] = 0u;
  if (local && !last)  // hs: the next pass's [dest tile][digit] counts of this tile
    for (int i = threadIdx.x; i < ntiles * R; i += NT) hs[i] = 0u;
  // every tile's counts of my 4 digits (4*tid..4*tid+3): the first HB tiles' loads are issued
  // now and land during the ranking below
  constexpr int HB = 16;
  const uint4 *Hq = reinterpret_cast<const uint4 *>(Hp) + threadIdx.x;
  uint4 hc[HB];
#pragma unroll
  for (int u = 0; u < HB; ++u) hc[u] = u < ntiles ? Hq[(int64_t)u * (R / 4)] : make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const bool valid = base + it * 64 < V;
    const uint32_t d = digit(key[it], pass);
    const uint64_t m = match_bits<BITS>(d, valid);
    const uint32_t r = valid ? wcnt[wv][d] : 0u;
    rk[it] = r + (uint32_t)__popcll(m & lt);
    if (valid && (m & lt) == 0) wcnt[wv][d] = r + (uint32_t)__popcll(m);
  }
  {
    constexpr int PER = R / NT;
    int tot[PER], before[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) tot[j] = before[j] = 0;
    auto acc = [&](const uint4 c, int u) {
      const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        tot[j] += (int)cc[j];
        before[j] += u < t ? (int)cc[j] : 0;
      }
    };
#pragma unroll
    for (int u = 0; u < HB; ++u) acc(hc[u], u);
    for (int u0 = HB; u0 < ntiles; u0 += HB) {
#pragma unroll
      for (int u = 0; u < HB; ++u)
        hc[u] = u0 + u < ntiles ? Hq[(int64_t)(u0 + u) * (R / 4)] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int u = 0; u < HB; ++u) acc(hc[u], u0 + u);
    }
    int sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) sum += tot[j];
    int off = block_excl_scan2<NT>(sum, wtot, nullptr);  // synchronises the block
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      gbase[PER * threadIdx.x + j] = (uint32_t)(off + before[j]);
      off += tot[j];
    }
  }
  __syncthreads();
  for (int dd = threadIdx.x; dd < R; dd += NT) {  // fold per-wave prefixes into the bases
    const uint32_t c0 = wcnt[0][dd], c1 = wcnt[1][dd], c2 = wcnt[2][dd];
    const uint32_t g = gbase[dd];
    wcnt[0][dd] = g;
    wcnt[1][dd] = g + c0;
    wcnt[2][dd] = g + c0 + c1;
    wcnt[3][dd] = g + c0 + c1 + c2;
  }
  __syncthreads();
  const int want = want_eff(rq, V);
  int32_t *adds, *nadd;
  float *addv, *cutv;
  outs_resolve(o, want, adds, nadd, addv, cutv);
  if (pass == 0 && t == 0) {
    const int n = req_n(rq);
    const int32_t *ids = req_ids(rq);
    for (int i = threadIdx.x; i < n; i += NT) cutv[i] = probs[ids[i]];
    if (threadIdx.x == 0) *nadd = want;
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    if (base + it * 64 >= V) continue;
    const uint32_t pos = wcnt[wv][digit(key[it], pass)] + rk[it];
    if (pos >= (uint32_t)V) continue;  // only reachable with inconsistent histograms: never write OOB
    if (last) {
      const int q = V - 1 - (int)pos;  // descending position
      if (q < want) {
        adds[q] = (int32_t)id[it];
        addv[q] = __uint_as_float(key[it] - 1u);
      }
    } else {
      kdst[pos] = key[it];
      idst[pos] = id[it];
      const uint32_t hi = (pos / TILE) * R + digit(key[it], pass + 1);
      if (local)
        atomicAdd(&hs[hi], 1u);
      else
        atomicAdd(&w.H[(int64_t)(pass + 1) * ntiles * R + hi], 1u);
    }
  }
  if (last || !local) return;
  __syncthreads();
  uint32_t *Hn = w.H + (int64_t)(pass + 1) * ntiles * R;
  for (int i = threadIdx.x; i < ntiles * R; i += NT) {
    const uint32_t c = hs[i];
    if (c) atomicAdd(&Hn[i], c);
  }
}

// Exclusive scan of hist[digit*FNW + wave] in place (digit-major: stable across waves).
__device__ __forceinline__ void scan_hist(uint32_t *hist, int *wtot) {
  constexpr int PER = RADIX * FNW / FNT;  // 4
  uint32_t loc[PER];
  int s = 0;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    loc[e] = hist[threadIdx.x * PER + e];
    s += (int)loc[e];
  }
  int off = block_excl_scan2<FNT>(s, wtot, nullptr);
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    hist[threadIdx.x * PER + e] = (uint32_t)off;
    off += (int)loc[e];
  }
}

// ------------------------------------------------------------------ full ranking (one workgroup)
__device__ __forceinline__ int block_excl_scan(int v, int *sc, int *total) {
  // sc: [FNT] scratch in LDS
  sc[threadIdx.x] = v;
  __syncthreads();
  for (int off = 1; off < FNT; off <<= 1) {
    const int t = threadIdx.x >= off ? sc[threadIdx.x - off] : 0;
    __syncthreads();
    sc[threadIdx.x] += t;
    __syncthreads();
  }
  const int incl = sc[threadIdx.x];
  if (total) *total = sc[FNT - 1];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(FNT) void topn_full_kernel(const float *__restrict__ probs, int V,
                                                         const int32_t *__restrict__ cube_idx,
                                                         int n, int amount, int32_t *additions,
                                                         int32_t *n_add, float *add_vals,
                                                         float *cut_vals, int32_t *order_out,
                                                         uint32_t *ws) {
  __shared__ uint32_t hist[RADIX * FNW];  // [digit][wave]
  __shared__ int sc[FNT];
  extern __shared__ __attribute__((aligned(16))) uint32_t cube_bits[];  // [ceil(V/32)]
  const int VW = (V + 31) >> 5;
  uint32_t *kA = ws, *kB = ws + V;
  int32_t *vA = (int32_t *)(ws + 2 * (int64_t)V), *vB = vA + V;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;

  for (int i = threadIdx.x; i < VW; i += FNT) cube_bits[i] = 0u;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += FNT) {
    const int j = cube_idx[i];
    atomicOr(&cube_bits[j >> 5], 1u << (j & 31));
    cut_vals[i] = probs[j];
  }

  const int S = (int)cdiv(cdiv(V, FNW), 64) * 64;  // per-wave slice
  const int lo = w * S, hi = min(V, lo + S);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    const uint32_t *ksrc = (pass & 1) ? kB : kA;
    const int32_t *vsrc = (pass & 1) ? vB : vA;
    uint32_t *kdst = (pass & 1) ? kA : kB;
    int32_t *vdst = (pass & 1) ? vA : vB;
    for (int i = threadIdx.x; i < RADIX * FNW; i += FNT) hist[i] = 0u;
    __syncthreads();
    for (int base = lo; base < hi; base += 64) {
      const int i = base + lane;
      const bool valid = i < hi;
      uint32_t key = 0;
      if (valid) key = pass == 0 ? __float_as_uint(probs[i]) : ksrc[i];
      const uint32_t dg = (key >> shift) & 0xFFu;
      const uint64_t m = match_digit(dg, valid);
      if (valid && (m & lt) == 0) hist[dg * FNW + w] += (uint32_t)__popcll(m);
    }
    __syncthreads();
    scan_hist(hist, sc);
    __syncthreads();
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
      if (valid) basepos = hist[dg * FNW + w];
      if (valid) {
        const uint32_t pos = basepos + (uint32_t)__popcll(m & lt);
        kdst[pos] = key;
        vdst[pos] = val;
      }
      if (valid && (m & lt) == 0) hist[dg * FNW + w] = basepos + (uint32_t)__popcll(m);
    }
    __threadfence_block();
    __syncthreads();
  }
  const int want = amount > 0 ? amount : 1;
  int done = 0;
  for (int q0 = 0; q0 < V && done < want; q0 += FNT) {
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
    for (int q = threadIdx.x; q < V; q += FNT) order_out[q] = vA[V - 1 - q];
  if (threadIdx.x == 0) *n_add = done < want ? done : want;
}


}  // namespace

extern "C" size_t cc_topn_workspace_size(int32_t V) {
  const size_t v = (size_t)std::max(V, 1);
  return std::max(tiles::ws_bytes((int)v), 4 * (4 * v + 16));
}

namespace cc {
int topn_tile_passes(int V, void *ws, const float *probs, tiles::Req rq, tiles::Outs o,
                     hipStream_t s) {
  const int nt = tiles::count(V);
  const tiles::Ws w = tiles::ws_of(ws, V);
  const size_t lds = nt <= tiles::LOCAL_TILES ? (size_t)nt * tiles::R * 4 : 0;
  for (int p = 0; p < tiles::PASSES; ++p) {
    hipLaunchKernelGGL(topn_pass_kernel, dim3(nt), dim3(tiles::NT), lds, s, p, V, nt, w, probs,
                       rq, o);
    CC_LAUNCH_CHECK("topn_pass_kernel");
  }
  return CC_OK;
}

int topn_launch(const float *probs, int V, const int32_t *cube_idx, int n, int amount,
                int32_t *additions, int32_t *n_add, float *add_vals, float *cut_vals,
                int32_t *order, void *ws, hipStream_t s) {
  if (order) {
    const size_t lds = (size_t)cdiv(V, 32) * 4;
    if (lds > 96 * 1024) return cc::fail(CC_ERR_UNSUPPORTED, "cc_topn: V too large for order");
    hipLaunchKernelGGL(topn_full_kernel, dim3(1), dim3(FNT), lds, s, probs, V, cube_idx, n, amount,
                       additions, n_add, add_vals, cut_vals, order, (uint32_t *)ws);
    CC_LAUNCH_CHECK("topn_full_kernel");
    return CC_OK;
  }
  const int nt = tiles::count(V);
  const tiles::Ws w = tiles::ws_of(ws, V);
  hipLaunchKernelGGL(topn_init_kernel, dim3(nt), dim3(tiles::NT), 0, s, probs, V, cube_idx, n, w,
                     nt);
  CC_LAUNCH_CHECK("topn_init_kernel");
  tiles::Req rq{nullptr, cube_idx, n, amount};
  tiles::Outs o{additions, n_add, add_vals, cut_vals, nullptr};
  return topn_tile_passes(V, ws, probs, rq, o, s);
}
}  // namespace cc

extern "C" int cc_topn(const float *probs, int32_t V, const int32_t *cube_idx, int32_t n,
                       int32_t amount, int32_t *additions, int32_t *n_additions, float *add_vals,
                       float *cut_vals, int32_t *order, void *ws, void *stream) {
  CC_REQUIRE(probs && additions && n_additions && add_vals && ws, "cc_topn: null pointer");
  CC_REQUIRE(V > 0 && n >= 0 && n <= V, "cc_topn: bad V/n");
  CC_REQUIRE(n == 0 || (cube_idx && cut_vals), "cc_topn: cube_idx/cut_vals needed when n > 0");
  return cc::topn_launch(probs, V, cube_idx, n, amount, additions, n_additions, add_vals,
                         cut_vals, order, ws, as_stream(stream));
}
