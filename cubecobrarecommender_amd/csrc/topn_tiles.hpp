// Shared pieces of the tiled top-N sort (topn.hip) and the recommend output layer (infer.hip),
// which produces the sort's keys and first digit histogram as it writes the probabilities.
//
// Sort key of card c:  key'(c) = in_cube(c) ? 0 : float_bits(prob_c) + 1   (prob in [0, 1], so
// key' < 2^30: three 10-bit LSD passes).  Ascending stable order of key' read backwards is the
// pinned ranking (descending prob, ties -> higher index) with the cube cards last.
#pragma once
#include "common.hpp"

namespace tiles {
constexpr int BITS = 10;
constexpr int R = 1 << BITS;   // digits per pass
constexpr int PASSES = 3;
constexpr int TILE = 1024;     // positions per tile workgroup
constexpr int NT = 256;        // threads per tile workgroup
constexpr int IT = TILE / NT;  // items per thread
constexpr int LOCAL_TILES = 32;  // up to this many tiles, histograms are staged in LDS

__host__ __device__ inline int count(int V) { return (V + TILE - 1) / TILE; }

__device__ __forceinline__ uint32_t digit(uint32_t key, int pass) {
  return (key >> (BITS * pass)) & (uint32_t)(R - 1);
}
__device__ __forceinline__ uint32_t key_of(float p, bool in_cube) {
  return in_cube ? 0u : __float_as_uint(p) + 1u;
}

// Workspace: keys/ids ping-pong [V] x 4, histograms H[PASSES][tiles][R], cube bitmask [V/32].
struct Ws {
  uint32_t *kA, *iA, *kB, *iB, *H, *bits;
};
__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
__host__ __device__ inline Ws ws_of(void *base, int V) {
  char *p = (char *)base;
  const size_t v = align256((size_t)V * 4);
  Ws w;
  w.kA = (uint32_t *)p;
  w.iA = (uint32_t *)(p + v);
  w.kB = (uint32_t *)(p + 2 * v);
  w.iB = (uint32_t *)(p + 3 * v);
  w.H = (uint32_t *)(p + 4 * v);
  w.bits = (uint32_t *)(p + 4 * v + align256((size_t)PASSES * count(V) * R * 4));
  return w;
}
inline size_t ws_bytes(int V) {
  return 4 * align256((size_t)V * 4) + align256((size_t)PASSES * count(V) * R * 4) +
         align256((size_t)(V + 31) / 32 * 4) + 256;
}
inline size_t zero_words(int V) {  // H + bits, contiguous
  return (align256((size_t)PASSES * count(V) * R * 4) + align256((size_t)(V + 31) / 32 * 4)) / 4;
}

// The request: device {n, amount, ids[n]} (req != nullptr) or host values.
struct Req {
  const int32_t *req;
  const int32_t *ids;  // used when req == nullptr
  int n, amount;
};
__device__ __forceinline__ int req_n(const Req &q) { return q.req ? q.req[0] : q.n; }
__device__ __forceinline__ int req_amount(const Req &q) { return q.req ? q.req[1] : q.amount; }
__device__ __forceinline__ const int32_t *req_ids(const Req &q) { return q.req ? q.req + 2 : q.ids; }
__device__ __forceinline__ int want_eff(const Req &q, int V) {
  const int a = req_amount(q);
  return min(a > 0 ? a : 1, V - req_n(q));
}

// Outputs: explicit pointers, or one packed buffer {n_add, additions[w], add_vals[w], cut[n]}.
struct Outs {
  int32_t *additions, *n_add;
  float *add_vals, *cut_vals;
  int32_t *packed;
};
__device__ __forceinline__ void outs_resolve(const Outs &o, int want, int32_t *&adds,
                                             int32_t *&nadd, float *&addv, float *&cutv) {
  if (o.packed) {
    nadd = o.packed;
    adds = o.packed + 1;
    addv = reinterpret_cast<float *>(o.packed + 1 + want);
    cutv = reinterpret_cast<float *>(o.packed + 1 + 2 * want);
  } else {
    adds = o.additions;
    nadd = o.n_add;
    addv = o.add_vals;
    cutv = o.cut_vals;
  }
}
}  // namespace tiles

namespace cc {
// Launch the PASSES tile passes (keys/ids in ws.kA/iA and H[0] already built, H[1..] zero).
int topn_tile_passes(int V, void *ws, const float *probs, tiles::Req rq, tiles::Outs o,
                     hipStream_t s);
}
