// Recommend forward pass in fp32 with a PINNED summation order — bit-exact against
// oracle/infer_ref.py.  Replaces `model.encoder(x)` / `model.decoder(z)` of
// src/scripts/ml_recommend.py:78-85 and web/ml_recommend_web.py:39-44.
//
// Pinned arithmetic (every multiply and add separately rounded: contraction is off here):
//   E1:   sorted unique card ids in chunks of 32; each chunk summed from 0 in order; chunk sums
//         added in order from 0; + bias; ReLU = (x > 0 ? x : 0).
//   Dense: K in chunks of 64; chunk acc = acc + h[k]*W[k][c] from 0; chunk partials added in
//          order from 0; + bias; ReLU.
//   Output: same dot, then sigmoid = float(1/(1+exp(-z))) in fp64 with the deterministic exp.
//
// A single-cube request is latency-bound (~45 MB of weights, MALL-resident after the first
// request), so every kernel is shaped for memory-level parallelism: each thread owns whole
// summation chains and issues all of a chain's loads before its first add.
//   gather_partials_kernel: one workgroup per (chunk of 32 cards, cube); float4 columns.
//   tower_kernel:           one workgroup per cube: chunk sums + bias (E1), then the Dense layers
//                           of the encoder and/or decoder tower with activations in LDS.
//   out_kernel:             one wave per 64-wide K chunk, 64 cards per workgroup; the chunk
//                           partials meet in LDS and wave 0 adds them in order + sigmoid.
#include "common.hpp"
#include "detmath.hpp"
#include "topn_tiles.hpp"

namespace {

constexpr int NT = 1024;  // tower workgroup
constexpr int GCH = 32;   // gather chunk (rows)
constexpr int GNT = 128;  // gather workgroup
constexpr int KCH = 64;   // dot chunk

struct Layer {
  const float *W, *b;
  int K, N;
};
struct Tower {
  const float *W1, *b1;  // E1 (gather)
  Layer L[6];            // encoder e2,e3,bottleneck, decoder d1,d2,d3
  int d;
};

__device__ __forceinline__ float addf(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float mulf(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(addf(a.x, b.x), addf(a.y, b.y), addf(a.z, b.z), addf(a.w, b.w));
}

// part[r][c][:] = sum_{j in chunk c of row r} W1[idx[j]][:]   (sequential from 0)
// row_ptr == nullptr: a single row, the request's ids (tiles::Req).  zero/nzero: words the
// request path clears for the top-N sort (its histograms and cube bitmask), grid-strided.
__global__ __launch_bounds__(GNT) void gather_partials_kernel(const float *__restrict__ W1, int d,
                                                              const int32_t *__restrict__ row_ptr,
                                                              const int32_t *__restrict__ idx,
                                                              tiles::Req rq, int cap,
                                                              float *__restrict__ part,
                                                              uint32_t *zero, int64_t nzero) {
  __shared__ int32_t lst[GCH];
  for (int64_t i = (int64_t)blockIdx.x * GNT + threadIdx.x; i < nzero / 4;
       i += (int64_t)gridDim.x * GNT)
    reinterpret_cast<uint4 *>(zero)[i] = make_uint4(0u, 0u, 0u, 0u);
  const int r = blockIdx.y;
  const int beg = row_ptr ? row_ptr[r] : 0;
  const int n = row_ptr ? row_ptr[r + 1] - beg : tiles::req_n(rq);
  const int32_t *ids = row_ptr ? idx : tiles::req_ids(rq);
  const int nch = (n + GCH - 1) / GCH;
  for (int c = blockIdx.x; c < nch; c += gridDim.x) {
    const int j0 = c * GCH, cnt = min(GCH, n - j0);
    __syncthreads();
    if (threadIdx.x < GCH) lst[threadIdx.x] = threadIdx.x < cnt ? ids[beg + j0 + threadIdx.x] : 0;
    __syncthreads();
    float *out = part + ((int64_t)r * cap + c) * d;
    for (int c4 = threadIdx.x; c4 < d / 4; c4 += GNT) {
      float4 v[GCH];
#pragma unroll
      for (int j = 0; j < GCH; ++j)
        if (j < cnt) v[j] = *reinterpret_cast<const float4 *>(W1 + (int64_t)lst[j] * d + 4 * c4);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < GCH; ++j)
        if (j < cnt) acc = add4(acc, v[j]);
      *reinterpret_cast<float4 *>(out + 4 * c4) = acc;
    }
  }
}

// out[n] = relu?(blocked_dot(h, W[:, n]) + b[n]); scratch = [K/KCH][N] floats.  K % 64 == 0.
__device__ void dense_lds(const float *h, const Layer &L, float *out, float *scratch, bool do_relu) {
  const int nch = L.K / KCH;
  for (int t = threadIdx.x; t < nch * L.N; t += NT) {
    const int c = t / L.N, n = t % L.N;
    const float *Wp = L.W + (int64_t)c * KCH * L.N + n;
    float w[KCH];
#pragma unroll
    for (int k = 0; k < KCH; ++k) w[k] = Wp[(int64_t)k * L.N];
    const float *hc = h + c * KCH;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < KCH; ++k) acc = addf(acc, mulf(hc[k], w[k]));
    scratch[t] = acc;
  }
  __syncthreads();
  for (int n = threadIdx.x; n < L.N; n += NT) {
    float tot = 0.f;
    for (int c = 0; c < nch; ++c) tot = addf(tot, scratch[c * L.N + n]);
    const float v = addf(tot, L.b[n]);
    out[n] = do_relu ? relu(v) : v;
  }
  __syncthreads();
}

// mode 0: encode (E1 from chunk partials + e2,e3,bottleneck) -> out = zlat [R,64]
// mode 1: decode tower (d1,d2,d3) from zin [R,64]           -> out = h3 [R,d]
// mode 2: both                                              -> zlat_out [R,64] and out = h3
__global__ __launch_bounds__(NT) void tower_kernel(Tower T, int mode,
                                                   const int32_t *__restrict__ row_ptr,
                                                   tiles::Req rq, uint32_t *cube_bits,
                                                   const float *__restrict__ part, int cap,
                                                   const float *__restrict__ zin,
                                                   float *__restrict__ zlat_out,
                                                   float *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int d = T.d;
  float *hA = sm;              // [1024]
  float *hB = hA + 1024;       // [1024]
  float *scratch = hB + 1024;  // [max over layers of K/KCH*N]
  const int r = blockIdx.x;
  if (mode == 2 && cube_bits) {  // the request's cube bitmask (zeroed by the gather kernel)
    const int n = tiles::req_n(rq);
    const int32_t *ids = tiles::req_ids(rq);
    for (int i = threadIdx.x; i < n; i += NT) atomicOr(&cube_bits[ids[i] >> 5], 1u << (ids[i] & 31));
  }
  if (mode != 1) {
    const int n = row_ptr ? row_ptr[r + 1] - row_ptr[r] : tiles::req_n(rq);
    const int nch = (n + GCH - 1) / GCH;
    const float *pr = part + (int64_t)r * cap * d;
    for (int col = threadIdx.x; col < d; col += NT) {
      float tot = 0.f;
      for (int c = 0; c < nch; ++c) tot = addf(tot, pr[(int64_t)c * d + col]);
      hA[col] = relu(addf(tot, T.b1[col]));
    }
    __syncthreads();
    dense_lds(hA, T.L[0], hB, scratch, true);
    dense_lds(hB, T.L[1], hA, scratch, true);
    dense_lds(hA, T.L[2], hB, scratch, true);
    if (mode == 0) {
      for (int c = threadIdx.x; c < 64; c += NT) out[(int64_t)r * 64 + c] = hB[c];
      return;
    }
    for (int c = threadIdx.x; c < 64; c += NT) {
      zlat_out[(int64_t)r * 64 + c] = hB[c];
      hA[c] = hB[c];
    }
    __syncthreads();
  } else {
    for (int c = threadIdx.x; c < 64; c += NT) hA[c] = zin[(int64_t)r * 64 + c];
    __syncthreads();
  }
  dense_lds(hA, T.L[3], hB, scratch, true);
  dense_lds(hB, T.L[4], hA, scratch, true);
  dense_lds(hA, T.L[5], hB, scratch, true);
  for (int c = threadIdx.x; c < d; c += NT) out[(int64_t)r * d + c] = hB[c];
}

// probs[r][n] = sigmoid(blocked_dot(h3[r], Wo[:, n]) + bo[n]); blockDim = (d/64) waves.
// sort != nullptr (single-cube request): also emits the top-N sort's keys/ids and pass-0 digit
// counts (tiles::key_of with the cube bitmask).
__global__ __launch_bounds__(1024) void out_kernel(const float *__restrict__ h3,
                                                   const float *__restrict__ Wo,
                                                   const float *__restrict__ bo, int d, int V,
                                                   float *__restrict__ probs, tiles::Ws sort,
                                                   int with_sort) {
  __shared__ float part[16][64];
  __shared__ float hs[1024];
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = d / KCH;
  const int r = blockIdx.y;
  const int n = blockIdx.x * 64 + lane;
  hs[threadIdx.x] = h3[(int64_t)r * d + threadIdx.x];  // blockDim == d
  __syncthreads();
  if (n < V) {
    const float *Wp = Wo + (int64_t)c * KCH * V + n;
    float w[KCH];
#pragma unroll
    for (int k = 0; k < KCH; ++k) w[k] = Wp[(int64_t)k * V];
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < KCH; ++k) acc = addf(acc, mulf(hs[c * KCH + k], w[k]));
    part[c][lane] = acc;
  }
  __syncthreads();
  if (c == 0 && n < V) {
    float tot = 0.f;
    for (int cc = 0; cc < nch; ++cc) tot = addf(tot, part[cc][lane]);
    const float p = detm::det_sigmoid32(addf(tot, bo[n]));
    probs[(int64_t)r * V + n] = p;
    if (with_sort) {
      const uint32_t key = tiles::key_of(p, (sort.bits[n >> 5] >> (n & 31)) & 1u);
      sort.kA[n] = key;
      sort.iA[n] = (uint32_t)n;
      atomicAdd(&sort.H[(int64_t)(n / tiles::TILE) * tiles::R + tiles::digit(key, 0)], 1u);
    }
  }
}

int tower_lds_bytes(int d) {
  int scratch = 0;
  const int shapes[6][2] = {{d, 256}, {256, 128}, {128, 64}, {64, 128}, {128, 256}, {256, d}};
  for (auto &s : shapes) scratch = std::max(scratch, (s[0] / KCH) * s[1]);
  return (2048 + scratch) * 4;
}

}  // namespace

// layout helper implemented in api.cpp
namespace cc {
int param_offsets(int V, int d, int64_t *off, int64_t *size, int64_t *total, int64_t *main_total);
int topn_launch(const float *probs, int V, const int32_t *cube_idx, int n, int amount,
                int32_t *additions, int32_t *n_add, float *add_vals, float *cut_vals,
                int32_t *order, void *ws, hipStream_t stream);
}

static int make_tower(const float *params, int V, int d, Tower &T) {
  int64_t off[CC_NUM_TENSORS], sz[CC_NUM_TENSORS], tot, mt;
  int rc = cc::param_offsets(V, d, off, sz, &tot, &mt);
  if (rc) return rc;
  T.d = d;
  T.W1 = params + off[0];
  T.b1 = params + off[1];
  // tensor indices: encoder e1..bottleneck = 0..7, decoder d1..reconstruct = 8..15
  const int ti[6] = {2, 4, 6, 8, 10, 12};
  const int Ks[6] = {d, 256, 128, 64, 128, 256};
  const int Ns[6] = {256, 128, 64, 128, 256, d};
  for (int l = 0; l < 6; ++l) {
    T.L[l].W = params + off[ti[l]];
    T.L[l].b = params + off[ti[l] + 1];
    T.L[l].K = Ks[l];
    T.L[l].N = Ns[l];
  }
  return CC_OK;
}

static int check_d(int d, const char *who) {
  if (!(d >= 64 && d <= 1024 && d % 64 == 0))
    return cc::fail(CC_ERR_ARG, std::string(who) + ": d must be a multiple of 64 in [64, 1024]");
  return CC_OK;
}

static inline int gather_cap(int max_n) { return std::max(1, (int)cdiv(std::max(max_n, 0), GCH)); }

extern "C" size_t cc_infer_encode_ws_size(int32_t R, int32_t d, int32_t max_n) {
  return (size_t)std::max(R, 1) * gather_cap(max_n) * std::max(d, 64) * sizeof(float);
}

extern "C" int cc_infer_encode_fp32(const float *params, int32_t V, int32_t d, int32_t R,
                                    const int32_t *row_ptr, const int32_t *idx, int32_t max_n,
                                    void *ws, float *zlat, void *stream) {
  CC_REQUIRE(params && row_ptr && idx && zlat && ws, "cc_infer_encode_fp32: null pointer");
  if (int rc = check_d(d, "cc_infer_encode_fp32")) return rc;
  CC_REQUIRE(max_n >= 0 && max_n <= V, "cc_infer_encode_fp32: max_n");
  if (R == 0) return CC_OK;
  Tower T;
  if (int rc = make_tower(params, V, d, T)) return rc;
  const int cap = gather_cap(max_n);
  float *part = (float *)ws;
  hipStream_t s = as_stream(stream);
  const tiles::Req none{nullptr, nullptr, 0, 0};
  hipLaunchKernelGGL(gather_partials_kernel, dim3(std::min(cap, 64), R), dim3(GNT), 0, s, T.W1, d,
                     row_ptr, idx, none, cap, part, (uint32_t *)nullptr, (int64_t)0);
  CC_LAUNCH_CHECK("gather_partials_kernel");
  hipLaunchKernelGGL(tower_kernel, dim3(R), dim3(NT), tower_lds_bytes(d), s, T, 0, row_ptr, none,
                     (uint32_t *)nullptr, (const float *)part, cap, (const float *)nullptr,
                     (float *)nullptr, zlat);
  CC_LAUNCH_CHECK("tower_kernel(encode)");
  return CC_OK;
}

extern "C" int cc_infer_decode_fp32(const float *params, int32_t V, int32_t d, int32_t R,
                                    const float *zlat, float *h3_ws, float *probs, void *stream) {
  CC_REQUIRE(params && zlat && h3_ws && probs, "cc_infer_decode_fp32: null pointer");
  if (int rc = check_d(d, "cc_infer_decode_fp32")) return rc;
  if (R == 0) return CC_OK;
  Tower T;
  if (int rc = make_tower(params, V, d, T)) return rc;
  hipStream_t s = as_stream(stream);
  const tiles::Req none{nullptr, nullptr, 0, 0};
  hipLaunchKernelGGL(tower_kernel, dim3(R), dim3(NT), tower_lds_bytes(d), s, T, 1,
                     (const int32_t *)nullptr, none, (uint32_t *)nullptr, (const float *)nullptr, 0,
                     zlat, (float *)nullptr, h3_ws);
  CC_LAUNCH_CHECK("tower_kernel(decode)");
  int64_t off[CC_NUM_TENSORS], sz[CC_NUM_TENSORS], tot, mt;
  if (int rc = cc::param_offsets(V, d, off, sz, &tot, &mt)) return rc;
  hipLaunchKernelGGL(out_kernel, dim3((unsigned)cdiv(V, 64), R), dim3(d), 0, s, h3_ws,
                     params + off[14], params + off[15], d, V, probs, tiles::Ws{}, 0);
  CC_LAUNCH_CHECK("out_kernel");
  return CC_OK;
}

// ---------------------------------------------------------------------- single-cube request
// ws layout: [partials gather_cap(V)*d floats][zlat 64][h3 d] | top-N sort workspace
static size_t req_float_part(int V, int d) {
  return tiles::align256(((size_t)gather_cap(V) * d + 64 + d) * sizeof(float));
}

extern "C" size_t cc_recommend_ws_size(int32_t V, int32_t d) {
  return req_float_part(V, std::max(d, 64)) + tiles::ws_bytes(std::max(V, 1)) + 256;
}

// Fixed grids and no host-side dependence on the request: the launch sequence is replayable
// as a hipGraph with the request read from `req` on the device.
static int recommend_launch(const float *params, int V, int d, const int32_t *req, int max_n,
                            void *ws, float *probs, int32_t *res, hipStream_t s) {
  Tower T;
  if (int rc = make_tower(params, V, d, T)) return rc;
  int64_t off[CC_NUM_TENSORS], sz[CC_NUM_TENSORS], tot, mt;
  if (int rc = cc::param_offsets(V, d, off, sz, &tot, &mt)) return rc;
  const int cap = gather_cap(V);
  float *part = (float *)ws;
  float *zlat = part + (size_t)cap * d;
  float *h3 = zlat + 64;
  void *sws = (char *)ws + req_float_part(V, d);
  const tiles::Ws w = tiles::ws_of(sws, V);
  const tiles::Req rq{req, nullptr, 0, 0};
  const int gx = 64;  // chunk loop + clearing of the sort's histograms/bitmask, grid-strided
  (void)max_n;
  hipLaunchKernelGGL(gather_partials_kernel, dim3(gx, 1), dim3(GNT), 0, s, T.W1, d,
                     (const int32_t *)nullptr, (const int32_t *)nullptr, rq, cap, part, w.H,
                     (int64_t)tiles::zero_words(V));
  CC_LAUNCH_CHECK("gather_partials_kernel");
  hipLaunchKernelGGL(tower_kernel, dim3(1), dim3(NT), tower_lds_bytes(d), s, T, 2,
                     (const int32_t *)nullptr, rq, w.bits, (const float *)part, cap,
                     (const float *)nullptr, zlat, h3);
  CC_LAUNCH_CHECK("tower_kernel(recommend)");
  hipLaunchKernelGGL(out_kernel, dim3((unsigned)cdiv(V, 64), 1), dim3(d), 0, s, h3,
                     params + off[14], params + off[15], d, V, probs, w, 1);
  CC_LAUNCH_CHECK("out_kernel");
  const tiles::Outs o{nullptr, nullptr, nullptr, nullptr, res};
  return cc::topn_tile_passes(V, sws, probs, rq, o, s);
}

extern "C" int cc_recommend_fp32(const float *params, int32_t V, int32_t d, const int32_t *req,
                                 int32_t max_n, void *ws, float *probs, int32_t *res,
                                 void *stream) {
  CC_REQUIRE(params && req && ws && probs && res, "cc_recommend_fp32: null pointer");
  CC_REQUIRE(V > 0 && max_n >= 0 && max_n <= V, "cc_recommend_fp32: V/max_n");
  if (int rc = check_d(d, "cc_recommend_fp32")) return rc;
  CC_REQUIRE(((uintptr_t)ws & 255) == 0, "cc_recommend_fp32: ws must be 256-byte aligned");
  return recommend_launch(params, V, d, req, max_n, ws, probs, res, as_stream(stream));
}

// ---------------------------------------------------------------------- request graph
// One request = [H2D of the request block] + the kernels above, captured once as a hipGraph;
// cc_recommend_graph_run replays it and copies back exactly the result words the caller asks
// for, so a request costs one graph launch + one D2H + one stream sync on the host.
struct cc_recommend_graph {
  hipStream_t stream;
  hipGraph_t graph;
  hipGraphExec_t exec;
  const int32_t *res_dev;
};

extern "C" int cc_recommend_graph_create(const float *params, int32_t V, int32_t d,
                                         const int32_t *req_host, int32_t *req_dev,
                                         int32_t max_n, void *ws, float *probs, int32_t *res_dev,
                                         void **handle) {
  CC_REQUIRE(params && req_host && req_dev && ws && probs && res_dev && handle,
             "cc_recommend_graph_create: null pointer");
  CC_REQUIRE(V > 0 && max_n >= 0 && max_n <= V, "cc_recommend_graph_create: V/max_n");
  if (int rc = check_d(d, "cc_recommend_graph_create")) return rc;
  CC_REQUIRE(((uintptr_t)ws & 255) == 0, "cc_recommend_graph_create: ws must be 256-byte aligned");
  auto *g = new cc_recommend_graph();
  g->res_dev = res_dev;
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    delete g;
    return cc::fail(CC_ERR_HIP, "cc_recommend_graph_create: stream");
  }
  hipError_t e = hipStreamBeginCapture(g->stream, hipStreamCaptureModeThreadLocal);
  int rc = CC_OK;
  if (e == hipSuccess) {
    e = hipMemcpyAsync(req_dev, req_host, (size_t)(2 + max_n) * sizeof(int32_t),
                       hipMemcpyHostToDevice, g->stream);
    if (e == hipSuccess) rc = recommend_launch(params, V, d, req_dev, max_n, ws, probs, res_dev, g->stream);
    hipError_t e2 = hipStreamEndCapture(g->stream, &g->graph);
    if (e == hipSuccess) e = e2;
  }
  if (e == hipSuccess && rc == CC_OK) e = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
  if (e != hipSuccess || rc != CC_OK) {
    hipStreamDestroy(g->stream);
    delete g;
    return rc != CC_OK ? rc : cc::fail(CC_ERR_HIP, std::string("cc_recommend_graph_create: ") + hipGetErrorString(e));
  }
  *handle = g;
  return CC_OK;
}

extern "C" int cc_recommend_graph_run(void *handle, int32_t *res_host, int32_t res_words) {
  CC_REQUIRE(handle && res_host && res_words >= 1, "cc_recommend_graph_run: bad argument");
  auto *g = (cc_recommend_graph *)handle;
  CC_HIP(hipGraphLaunch(g->exec, g->stream));
  CC_HIP(hipMemcpyAsync(res_host, g->res_dev, (size_t)res_words * sizeof(int32_t),
                        hipMemcpyDeviceToHost, g->stream));
  CC_HIP(hipStreamSynchronize(g->stream));
  return CC_OK;
}

extern "C" int cc_recommend_graph_destroy(void *handle) {
  if (!handle) return CC_OK;
  auto *g = (cc_recommend_graph *)handle;
  hipGraphExecDestroy(g->exec);
  hipGraphDestroy(g->graph);
  hipStreamDestroy(g->stream);
  delete g;
  return CC_OK;
}
