// N4: card similarity — src/scripts/similarity.py:19-31.
//
// The reference encodes the identity (model.encoder(I[V,V]) -> embs [V,64]), scores every card
// against the query with Keras CosineSimilarity (-sum(l2_normalize(a) * l2_normalize(b)),
// l2_normalize(x) = x * rsqrt(max(sum(x^2), 1e-12))) and prints the N smallest by argsort.
// Here the embeddings come from cc_infer_encode_fp32 on one-card rows; this file scores and ranks:
//
//   cosine_dist_kernel : one thread per card, fp32, multiply and add separately rounded in index
//                        order (no contraction): ss = sum e^2; inv = 1/sqrt(max(ss, 1e-12));
//                        dist_j = -(sum_i (q_i inv_q)(e_ji inv_j)).  Sort key = (orderable(dist)
//                        << 32) | j with -0 folded into +0: ascending key == numpy
//                        argsort(dist, kind='stable') (ties -> lower index first; the reference's
//                        default argsort leaves tie order implementation-defined).
//   rank_smallest_kernel: one 1024-thread workgroup: 8-bit radix SELECT of the N-th smallest
//                        64-bit key over all V keys (8 passes of LDS histograms), then the <= N
//                        selected keys bitonic-sorted in LDS.  Keys are unique, so exactly N.
#include "common.hpp"

namespace {

constexpr int SIM_NT = 1024;
constexpr int SIM_NMAX = 4096;  // N <= 4096 (the LDS sort)

__device__ __forceinline__ uint32_t orderable(float f) {
  uint32_t u = __float_as_uint(f == 0.f ? 0.f : f);  // -0 == +0 for the ranking
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void cosine_dist_kernel(const float *__restrict__ emb, int V, int K,
                                                          int q, float *__restrict__ dist,
                                                          uint64_t *__restrict__ keys) {
#pragma clang fp contract(off)
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= V) return;
  const float *e = emb + (int64_t)j * K, *qe = emb + (int64_t)q * K;
  float ssq = 0.f, sse = 0.f;
  for (int i = 0; i < K; ++i) {
    ssq = ssq + qe[i] * qe[i];
    sse = sse + e[i] * e[i];
  }
  const float invq = 1.f / sqrtf(fmaxf(ssq, 1e-12f)), inve = 1.f / sqrtf(fmaxf(sse, 1e-12f));
  float dot = 0.f;
  for (int i = 0; i < K; ++i) dot = dot + (qe[i] * invq) * (e[i] * inve);
  const float dd = -dot;
  dist[j] = dd;
  keys[j] = ((uint64_t)orderable(dd) << 32) | (uint32_t)j;
}

__global__ __launch_bounds__(SIM_NT) void rank_smallest_kernel(const uint64_t *__restrict__ keys,
                                                               const float *__restrict__ dist, int V,
                                                               int N, int32_t *__restrict__ out_idx,
                                                               float *__restrict__ out_dist) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_prefix, s_mask;
  __shared__ int s_remaining, s_cnt;
  __shared__ uint64_t sel[SIM_NMAX];
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_prefix = 0;
    s_mask = 0;
    s_remaining = N;
    s_cnt = 0;
  }
  __syncthreads();
  for (int pass = 7; pass >= 0; --pass) {
    for (int b = tid; b < 256; b += SIM_NT) hist[b] = 0u;
    __syncthreads();
    const uint64_t prefix = s_prefix, mask = s_mask;
    for (int j = tid; j < V; j += SIM_NT) {
      const uint64_t k = keys[j];
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> (8 * pass)) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {  // smallest digit whose cumulative count reaches the remaining rank
      int rem = s_remaining, dg = 0;
      for (; dg < 255 && (int)hist[dg] < rem; ++dg) rem -= (int)hist[dg];
      s_remaining = rem;
      s_prefix = prefix | ((uint64_t)dg << (8 * pass));
      s_mask = mask | ((uint64_t)255u << (8 * pass));
    }
    __syncthreads();
  }
  const uint64_t T = s_prefix;  // the N-th smallest key
  for (int j = tid; j < V; j += SIM_NT) {
    const uint64_t k = keys[j];
    if (k <= T) sel[atomicAdd(&s_cnt, 1)] = k;
  }
  __syncthreads();
  int P = 1;
  while (P < N) P <<= 1;
  for (int i = N + tid; i < P; i += SIM_NT) sel[i] = ~0ull;
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P; i += SIM_NT) {
        const int pr = i ^ stride;
        if (pr > i) {
          const bool up = (i & size) == 0;
          const uint64_t a = sel[i], b = sel[pr];
          if ((a > b) == up) {
            sel[i] = b;
            sel[pr] = a;
          }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < N; i += SIM_NT) {
    const int j = (int)(uint32_t)sel[i];
    out_idx[i] = j;
    out_dist[i] = dist[j];
  }
}

}  // namespace

extern "C" size_t cc_similar_ws_size(int32_t V) { return (size_t)V * (sizeof(uint64_t) + sizeof(float)) + 64; }

extern "C" int cc_similar_cards(const float *emb, int32_t V, int32_t K, int32_t q, int32_t N,
                                int32_t *out_idx, float *out_dist, float *dist_all, void *ws,
                                void *stream) {
  CC_REQUIRE(emb && out_idx && out_dist && ws, "cc_similar_cards: null pointer");
  CC_REQUIRE(V > 0 && K > 0 && q >= 0 && q < V, "cc_similar_cards: bad V/K/query");
  CC_REQUIRE(N >= 1 && N <= V && N <= SIM_NMAX, "cc_similar_cards: N must be 1..min(V, 4096)");
  CC_REQUIRE(((uintptr_t)ws & 7) == 0, "cc_similar_cards: ws must be 8-B aligned");
  uint64_t *keys = reinterpret_cast<uint64_t *>(ws);
  float *dist = dist_all ? dist_all : reinterpret_cast<float *>(keys + V);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(cosine_dist_kernel, dim3((unsigned)cdiv(V, 256)), dim3(256), 0, s, emb, V, K, q, dist, keys);
  CC_LAUNCH_CHECK("cosine_dist_kernel");
  hipLaunchKernelGGL(rank_smallest_kernel, dim3(1), dim3(SIM_NT), 0, s, keys, dist, V, N, out_idx, out_dist);
  CC_LAUNCH_CHECK("rank_smallest_kernel");
  return CC_OK;
}
