// Keras' compiled metrics=['accuracy'] of the reference's two outputs (train.py:83-88), counted
// on the device per step when the trainer runs with TrainConfig(metrics=True).  TF 2.5 resolves the
// string 'accuracy' per output by SHAPE, not by loss (keras/engine/compile_utils.py,
// MetricsContainer._get_metric_object): binary_accuracy only when y_pred's last dim is 1, sparse
// categorical when y_true has a lower rank, else categorical_accuracy.  Both outputs here are
// [B, |V|] against [B, |V|] targets, so BOTH are categorical_accuracy =
// mean over rows of [argmax(y_true) == argmax(y_pred)] (tf.argmax: first index on ties):
//   output_1 (sigmoid): y_pred = sigmoid(z) in fp32.  Eigen's float logistic (TF 2.5's CPU kernel)
//            saturates to exactly 1.0 from z >= 15.7243833541870117 on, so saturated logits tie and
//            the first one wins; below that the fp32 sigmoid is taken (ties there need two logits
//            within an fp32 rounding of each other).  y_true = the noised target row (0/1): its
//            argmax is its first set bit, 0 for an all-zero row;
//   output_2 (softmax): argmax(softmax(z)) = argmax(z) (first index on ties), y_true the row's M~
//            target (argmax precomputed once per M~ by cc_row_argmax).
// Counts are integers added with one atomic per block: the totals are order-free (deterministic).
// Off the training step's path (the fused output-layer kernels never store their logits): the
// trainer recomputes the logits for the metrics with cc_gemm from the same bf16 / fp32 operands.
// Parity unpinned (TF absent): the published rule and formulas are restated, Eigen's rational
// sigmoid approximation below the cut-off is not.
#include "common.hpp"

namespace {

constexpr int MT = 256;

// first index of the row's maximum (NaN-free rows)
__device__ __forceinline__ void argmax_pair(float &v, int &i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

// the block's (first) argmax from every thread's running (v, idx); contains __syncthreads
__device__ int block_argmax_reduce(float v, int idx) {
  __shared__ float sv[MT / 64];
  __shared__ int si[MT / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float v2 = __shfl_xor(v, off);
    const int i2 = __shfl_xor(idx, off);
    argmax_pair(v, idx, v2, i2);
  }
  if ((threadIdx.x & 63) == 0) {
    sv[threadIdx.x >> 6] = v;
    si[threadIdx.x >> 6] = idx;
  }
  __syncthreads();
  float bv = sv[0];
  int bi = si[0];
  for (int i = 1; i < MT / 64; ++i) argmax_pair(bv, bi, sv[i], si[i]);
  __syncthreads();
  return bi;
}

__device__ int block_argmax(const float *__restrict__ x, int V) {
  float v = -INFINITY;
  int idx = 0x7FFFFFFF;
  for (int j = threadIdx.x; j < V; j += MT) argmax_pair(v, idx, x[j], j);
  return block_argmax_reduce(v, idx);
}

__global__ __launch_bounds__(MT) void row_argmax_kernel(const float *__restrict__ X, int64_t ld, int V,
                                                        int32_t *__restrict__ out) {
  const int a = block_argmax(X + (int64_t)blockIdx.x * ld, V);
  if (threadIdx.x == 0) out[blockIdx.x] = a;
}

// rows with reg_idx >= 0 (padding rows are skipped): argmax(z row) == t_argmax[card - t_lo]
__global__ __launch_bounds__(MT) void cat_accuracy_kernel(const float *__restrict__ Z, int ldz, int V,
                                                          const int32_t *__restrict__ reg_idx,
                                                          const int32_t *__restrict__ t_argmax, int t_lo,
                                                          unsigned long long *__restrict__ count) {
  const int card = reg_idx[blockIdx.x];
  if (card < 0) return;   // (block-uniform)
  const int a = block_argmax(Z + (int64_t)blockIdx.x * ldz, V);
  if (threadIdx.x == 0) {
    atomicAdd(count + 1, 1ull);   // rows counted
    if (a == t_argmax[card - t_lo]) atomicAdd(count, 1ull);
  }
}


// Eigen scalar_logistic_op<float>: the rational approximation evaluates to exactly 1 from here on
constexpr float SIG_SAT = 15.7243833541870117f;
__device__ __forceinline__ float keras_sigmoid(float z) {
  return z >= SIG_SAT ? 1.0f : 1.0f / (1.0f + expf(-z));
}

// one block per batch row: [argmax_j sigmoid(z_j) == first set bit of the target row (0 if none)]
__global__ __launch_bounds__(MT) void sigmoid_cat_accuracy_kernel(const float *__restrict__ Z, int ldz,
                                                                  const uint32_t *__restrict__ y_bits, int V,
                                                                  unsigned long long *__restrict__ count) {
  __shared__ int sfirst[MT / 64];
  const int row = blockIdx.x, VW = (V + 31) >> 5;
  const float *z = Z + (int64_t)row * ldz;
  const uint32_t *y = y_bits + (int64_t)row * VW;
  int first = 0x7FFFFFFF;
  for (int w = threadIdx.x; w < VW; w += MT) {
    const uint32_t n = (uint32_t)min(32, V - 32 * w);
    const uint32_t bits = y[w] & (n == 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
    if (bits) first = min(first, 32 * w + __builtin_ctz(bits));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) first = min(first, __shfl_xor(first, off));
  if ((threadIdx.x & 63) == 0) sfirst[threadIdx.x >> 6] = first;
  float v = -INFINITY;
  int idx = 0x7FFFFFFF;
  for (int j = threadIdx.x; j < V; j += MT) argmax_pair(v, idx, keras_sigmoid(z[j]), j);
  const int a = block_argmax_reduce(v, idx);   // (its barrier also publishes sfirst)
  if (threadIdx.x == 0) {
    int t = sfirst[0];
    for (int i = 1; i < MT / 64; ++i) t = min(t, sfirst[i]);
    if (t == 0x7FFFFFFF) t = 0;   // tf.argmax of an all-zero row
    if (a == t) atomicAdd(count, 1ull);
  }
}

}  // namespace

extern "C" int cc_sigmoid_cat_accuracy(const float *Z, int32_t ldz, const uint32_t *y_bits, int32_t B, int32_t V,
                                       unsigned long long *count, void *stream) {
  CC_REQUIRE(Z && y_bits && count && B >= 0 && V > 0 && ldz >= V, "cc_sigmoid_cat_accuracy: args");
  if (B == 0) return CC_OK;
  hipLaunchKernelGGL(sigmoid_cat_accuracy_kernel, dim3((unsigned)B), dim3(MT), 0, as_stream(stream), Z, ldz, y_bits,
                     V, count);
  CC_LAUNCH_CHECK("sigmoid_cat_accuracy_kernel");
  return CC_OK;
}

extern "C" int cc_row_argmax(const float *X, int64_t ld, int32_t rows, int32_t V, int32_t *out, void *stream) {
  CC_REQUIRE(X && out && rows >= 0 && V > 0 && ld >= V, "cc_row_argmax: args");
  if (rows == 0) return CC_OK;
  hipLaunchKernelGGL(row_argmax_kernel, dim3((unsigned)rows), dim3(MT), 0, as_stream(stream), X, ld, V, out);
  CC_LAUNCH_CHECK("row_argmax_kernel");
  return CC_OK;
}

extern "C" int cc_cat_accuracy(const float *Z, int32_t ldz, int32_t rows, int32_t V, const int32_t *reg_idx,
                               const int32_t *t_argmax, int32_t t_lo, unsigned long long *count, void *stream) {
  CC_REQUIRE(Z && reg_idx && t_argmax && count && rows >= 0 && V > 0 && ldz >= V && t_lo >= 0,
             "cc_cat_accuracy: args");
  if (rows == 0) return CC_OK;
  hipLaunchKernelGGL(cat_accuracy_kernel, dim3((unsigned)rows), dim3(MT), 0, as_stream(stream), Z, ldz, V, reg_idx,
                     t_argmax, t_lo, count);
  CC_LAUNCH_CHECK("cat_accuracy_kernel");
  return CC_OK;
}
