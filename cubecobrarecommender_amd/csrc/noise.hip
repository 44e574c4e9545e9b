// cc_noise_fwd — the DAE input-noise function F and regulariser-row sampling on the GPU.
//
// Replaces src/ml/generator.py:38-103 (DataGenerator.__getitem__ / generate_data).  One
// 256-thread workgroup per cube; every draw is a pure function of
// (seed, step, slot, kind, index, try) through Philox4x32-10, so the whole batch is
// deterministic and bit-identical to oracle/noise_ref.py::philox_noise_batch.
//
// Per cube (n sorted card ids, LDS bitmasks over V):
//   noise = clip(mean + std * BoxMuller, .05, .8)          generator.py:86-90
//   k     = int(n * noise)                                  :91
//   cut   : k draws w/ replacement from the includes        :92
//   ycut  : k//4 draws w/ replacement from the cut multiset :95
//   add   : k draws, rejection against the global CDF of neg_sampler until the card is not
//           in the cube (== the renormalised law of :93-94), exact fallback after 256 tries
//   x = (cube \ cut) U add  (sorted CSR row),  y = cube \ ycut  (bitmask)     :96-101
// The B reg rows (generator.py:47-51) are drawn by thread 0 of each block into rows B..2B-1
// (with_reg = 1), or — data parallel with M~ row-sharded — all ranks draw the global slots and
// each keeps the rows it owns (cc_reg_rows, owner computes).
#include <algorithm>

#include "adam.hpp"
#include "common.hpp"
#include "detmath.hpp"
#include "noise_dev.hpp"

namespace {

using namespace ccnoise;

// Owner-computes reg rows: thread t draws global slots t, t + NTO, ... (the one-process draw of
// slot s), ownership bits are ballot-counted per wave, a block scan orders them by slot, and the
// owned cards land as rows B + pos of x.  Slot s is handled by thread s % NTO in round s / NTO, so
// the order "round-major, then thread" is slot order.
constexpr int NTO = 1024;
__global__ __launch_bounds__(NTO) void reg_rows_kernel(cc_noise_args a) {
  __shared__ int wsum[NTO / 64];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t step = (uint32_t)a.state[0];
  const int XW = (a.xt_rows + 31) >> 5;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int s0 = 0; s0 < a.reg_slots; s0 += NTO) {
    const int s = s0 + tid;
    int j = -1;
    if (s < a.reg_slots) {
      const u32x4 o = rng(a.seed, step, (uint32_t)s, KIND_REG, 0, 0);
      j = search_right(a.cdf, a.V, u53(o.x, o.y), a.guide, a.guide_log2);
    }
    const bool own = j >= a.reg_lo && j < a.reg_hi;
    const uint64_t m = __ballot(own);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    int off = base_s;
    for (int w = 0; w < wv; ++w) off += wsum[w];
    const int pos = off + before;
    if (own) {
      if (pos < a.reg_cap) {
        const int r = a.B + pos;
        a.reg_idx[pos] = j;
        a.x_idx[(int64_t)r * a.x_cap] = j;
        a.x_cnt[r] = 1;
        if (a.xt_bits && r < a.xt_rows) atomicOr(&a.xt_bits[(int64_t)j * XW + (r >> 5)], 1u << (r & 31));
      } else {
        atomicOr(a.status, 2);
      }
    }
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < NTO / 64; ++w) tot += wsum[w];
      base_s += tot;
    }
    __syncthreads();
  }
  // padding rows: masked (no KL term, zero gradient)
  for (int pos = base_s + tid; pos < a.reg_cap; pos += NTO) {
    a.reg_idx[pos] = -1;
    a.x_cnt[a.B + pos] = 0;
  }
}

__global__ __launch_bounds__(NT) void noise_kernel(cc_noise_args a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ int s_k;
  noise_block(a, smem, s_k, blockIdx.x, a.state[0], a.state[1], a.state[2]);
}

// Adam over the flat buffers in blocks [0, nadam) and, in blocks [nadam, nadam + B), F for the
// NEXT step (its {step, batch, epoch} = this step's advanced as cc_state_advance will): Adam is
// HBM-bound, F latency-bound, and F touches only the batch buffers this step's backward has
// released — one launch instead of F on the next step's critical path.
template <bool PACK>
__global__ __launch_bounds__(NT) void adam_noise_kernel(cc_adam::Args ad, cc_noise_args a,
                                                        int nadam, int64_t bpe, cc_adam::Pack pk,
                                                        cc_adam::Args ad1, int nadam1, int nf) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ int s_k;
  // F's nf (= B, or 0: Adam only) blocks come first: they are latency-bound chains that should
  // start at once, the Adam blocks (of the first flat range, then of the second, if any) stream
  // around them
  const int64_t step = a.state[0];
  if ((int)blockIdx.x >= nf + nadam) {
    cc_adam::range(ad1, step, (int)blockIdx.x - nf - nadam, nadam1, PACK ? &pk : nullptr);
  } else if ((int)blockIdx.x >= nf) {
    cc_adam::range(ad, step, (int)blockIdx.x - nf, nadam, PACK ? &pk : nullptr);
  } else {
    int64_t batch = a.state[1] + 1, epoch = a.state[2];
    if (batch >= bpe) {
      batch = 0;
      epoch += 1;
    }
    noise_block(a, smem, s_k, blockIdx.x, step + 1, batch, epoch);
  }
}

}  // namespace

static int noise_check(const cc_noise_args *a, size_t &lds) {
  CC_REQUIRE(a != nullptr && a->xt_rows >= a->B,
             "cc_noise_fwd: xt_rows must cover the cube rows (reg rows past xt_rows set no xt bit)");
  CC_REQUIRE(a != nullptr, "cc_noise_fwd: null args");
  CC_REQUIRE(a->V > 0 && a->B > 0 && a->x_cap > 0, "cc_noise_fwd: bad V/B/x_cap");
  CC_REQUIRE(a->cube_ptr && a->cube_idx && a->perm && a->cdf && a->neg_sampler && a->state,
             "cc_noise_fwd: null input pointer");
  CC_REQUIRE(a->x_cnt && a->x_idx && a->y_bits && a->status, "cc_noise_fwd: null output pointer");
  CC_REQUIRE(!a->with_reg || a->reg_idx, "cc_noise_fwd: with_reg needs reg_idx");
  CC_REQUIRE(a->num_perms >= 1 && a->num_cubes >= a->batch_stride, "cc_noise_fwd: num_perms/num_cubes");
  const int VW = (a->V + 31) / 32;
  lds = (size_t)(4 * VW + NT + 1) * 4;
  CC_REQUIRE(lds <= 150 * 1024, "cc_noise_fwd: V / x_cap too large for LDS");
  return CC_OK;
}

extern "C" int cc_noise_fwd(const cc_noise_args *a, void *stream) {
  size_t lds = 0;
  if (int rc = noise_check(a, lds)) return rc;
  hipLaunchKernelGGL(noise_kernel, dim3(a->B), dim3(NT), lds, as_stream(stream), *a);
  CC_LAUNCH_CHECK("noise_kernel");
  return CC_OK;
}

extern "C" int cc_reg_rows(const cc_noise_args *a, void *stream) {
  CC_REQUIRE(a != nullptr, "cc_reg_rows: null args");
  CC_REQUIRE(a->V > 0 && a->B > 0 && a->x_cap > 0 && a->reg_slots > 0 && a->reg_cap > 0,
             "cc_reg_rows: bad V/B/x_cap/reg_slots/reg_cap");
  CC_REQUIRE(a->reg_lo >= 0 && a->reg_lo < a->reg_hi && a->reg_hi <= a->V, "cc_reg_rows: shard [lo, hi)");
  CC_REQUIRE(a->cdf && a->state && a->x_cnt && a->x_idx && a->reg_idx && a->status,
             "cc_reg_rows: null pointer");
  CC_REQUIRE(!a->xt_bits || a->xt_rows >= a->B, "cc_reg_rows: xt_rows must cover the cube rows");
  hipLaunchKernelGGL(reg_rows_kernel, dim3(1), dim3(NTO), 0, as_stream(stream), *a);
  CC_LAUNCH_CHECK("reg_rows_kernel");
  return CC_OK;
}

extern "C" int cc_adam_noise(float *p, float *m, float *v, const float *g, uint16_t *shadow,
                             int64_t n, float lr, float beta1, float beta2, float eps,
                             const cc_noise_args *next, int64_t batches_per_epoch, void *stream) {
  CC_REQUIRE(p && m && v && g, "cc_adam_noise: null pointer");
  CC_REQUIRE(((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g) % 16 == 0,
             "cc_adam_noise: buffers must be 16-byte aligned");
  CC_REQUIRE(!shadow || (uintptr_t)shadow % 8 == 0, "cc_adam_noise: shadow must be 8-byte aligned");
  CC_REQUIRE(batches_per_epoch >= 1, "cc_adam_noise: batches_per_epoch");
  size_t lds = 0;
  if (int rc = noise_check(next, lds)) return rc;
  // one float4 per Adam thread (no grid-stride loop): the block dispatcher balances the Adam blocks
  // around F's latency-bound blocks (measured in step: 61 us vs 66-72 with a 2048-block grid)
  const int nadam = n > 0 ? (int)cdiv(cdiv(n, 4), NT) : 0;
  const cc_adam::Args ad{p, m, v, g, (bf16_t *)shadow, n, lr, beta1, beta2, eps};
  hipLaunchKernelGGL(adam_noise_kernel<false>, dim3((unsigned)(nadam + next->B)), dim3(NT), lds,
                     as_stream(stream), ad, *next, nadam, batches_per_epoch, cc_adam::Pack{}, cc_adam::Args{}, 0,
                     next->B);
  CC_LAUNCH_CHECK("adam_noise_kernel");
  return CC_OK;
}

extern "C" int cc_noise_next(const cc_noise_args *a, int64_t batches_per_epoch, void *stream) {
  CC_REQUIRE(batches_per_epoch >= 1, "cc_noise_next: batches_per_epoch");
  size_t lds = 0;
  if (int rc = noise_check(a, lds)) return rc;
  hipLaunchKernelGGL(adam_noise_kernel<false>, dim3((unsigned)a->B), dim3(NT), lds, as_stream(stream),
                     cc_adam::Args{}, *a, 0, batches_per_epoch, cc_adam::Pack{}, cc_adam::Args{}, 0, a->B);
  CC_LAUNCH_CHECK("adam_noise_kernel (F only)");
  return CC_OK;
}

static int adam_pack2_launch(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t lo0,
                             int64_t n0, int64_t lo1, int64_t n1, float lr, float beta1, float beta2, float eps,
                             const cc_noise_args *next, int64_t batches_per_epoch, const cc_adam_pack *pack,
                             bool with_f, void *stream) {
  CC_REQUIRE(p && m && v && g && shadow && pack, "cc_adam_noise_pack: null pointer");
  CC_REQUIRE(((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g) % 16 == 0 && lo0 % 4 == 0 && lo1 % 4 == 0,
             "cc_adam_noise_pack: buffers must be 16-byte aligned, range starts multiples of 4");
  CC_REQUIRE(lo0 >= 0 && n0 >= 0 && n1 >= 0 && (n1 == 0 || lo1 >= lo0 + n0), "cc_adam_noise_pack2: ranges");
  const int64_t n = n1 > 0 ? lo1 + n1 : lo0 + n0;  // the extent the pack's layers must lie in
  CC_REQUIRE((uintptr_t)shadow % 8 == 0, "cc_adam_noise_pack: shadow must be 8-byte aligned");
  CC_REQUIRE(batches_per_epoch >= 1, "cc_adam_noise_pack: batches_per_epoch");
  CC_REQUIRE(pack->n >= 1 && pack->n <= 9, "cc_adam_noise_pack: 1..9 layers");
  cc_adam::Pack pk{};
  pk.n = pack->n;
  pk.lo = INT64_MAX;
  pk.hi = 0;
  for (int l = 0; l < pack->n; ++l) {
    const int K = pack->K[l], N = pack->N[l];
    CC_REQUIRE(K % 32 == 0 && N % 32 == 0 && pack->off[l] % 4 == 0 && pack->off[l] >= 0 &&
                   pack->off[l] + (int64_t)K * N <= n && pack->wpf[l] && pack->wpb[l] &&
                   (((uintptr_t)pack->wpb[l]) & 7) == 0,
               "cc_adam_noise_pack: layer shape / offset / image");
    pk.K[l] = K;
    pk.N[l] = N;
    pk.off[l] = pack->off[l];
    pk.wpf[l] = (bf16_t *)pack->wpf[l];
    pk.wpb[l] = (bf16_t *)pack->wpb[l];
    pk.lo = std::min<int64_t>(pk.lo, pack->off[l]);
    pk.hi = std::max<int64_t>(pk.hi, pack->off[l] + (int64_t)K * N);
  }
  size_t lds = 0;
  if (int rc = noise_check(next, lds)) return rc;
  for (int l = 0; l < pack->n; ++l)  // every packed layer inside one of the two ranges
    CC_REQUIRE((pack->off[l] >= lo0 && pack->off[l] + (int64_t)pack->K[l] * pack->N[l] <= lo0 + n0) ||
                   (pack->off[l] >= lo1 && pack->off[l] + (int64_t)pack->K[l] * pack->N[l] <= lo1 + n1),
               "cc_adam_noise_pack2: a packed layer outside the Adam ranges");
  const int nadam = n0 > 0 ? (int)cdiv(cdiv(n0, 4), NT) : 0;
  const int nadam1 = n1 > 0 ? (int)cdiv(cdiv(n1, 4), NT) : 0;
  const cc_adam::Args ad{p + lo0, m + lo0, v + lo0, g + lo0, (bf16_t *)shadow + lo0, n0, lr, beta1, beta2, eps, lo0};
  const cc_adam::Args ad1{p + lo1, m + lo1, v + lo1, g + lo1, (bf16_t *)shadow + lo1, n1, lr, beta1, beta2, eps, lo1};
  const int nf = with_f ? next->B : 0;
  hipLaunchKernelGGL(adam_noise_kernel<true>, dim3((unsigned)(nadam + nadam1 + nf)), dim3(NT), with_f ? lds : 0,
                     as_stream(stream), ad, *next, nadam, batches_per_epoch, pk, ad1, nadam1, nf);
  CC_LAUNCH_CHECK("adam_noise_kernel (pack)");
  return CC_OK;
}

extern "C" int cc_adam_noise_pack2(float *p, float *m, float *v, const float *g, uint16_t *shadow,
                                   int64_t lo0, int64_t n0, int64_t lo1, int64_t n1, float lr, float beta1,
                                   float beta2, float eps, const cc_noise_args *next, int64_t batches_per_epoch,
                                   const cc_adam_pack *pack, void *stream) {
  return adam_pack2_launch(p, m, v, g, shadow, lo0, n0, lo1, n1, lr, beta1, beta2, eps, next, batches_per_epoch,
                           pack, true, stream);
}

// the same Adam ranges + packed tower images without F (the next step's F drawn elsewhere: the
// tower backward launch, cc_tower_bwd_chain_noise); `next` only describes the launch checks
extern "C" int cc_adam_pack2(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t lo0,
                             int64_t n0, int64_t lo1, int64_t n1, float lr, float beta1, float beta2, float eps,
                             const cc_noise_args *next, int64_t batches_per_epoch, const cc_adam_pack *pack,
                             void *stream) {
  return adam_pack2_launch(p, m, v, g, shadow, lo0, n0, lo1, n1, lr, beta1, beta2, eps, next, batches_per_epoch,
                           pack, false, stream);
}

extern "C" int cc_adam_noise_pack(float *p, float *m, float *v, const float *g, uint16_t *shadow,
                                  int64_t n, float lr, float beta1, float beta2, float eps,
                                  const cc_noise_args *next, int64_t batches_per_epoch,
                                  const cc_adam_pack *pack, void *stream) {
  return cc_adam_noise_pack2(p, m, v, g, shadow, 0, n, 0, 0, lr, beta1, beta2, eps, next, batches_per_epoch,
                             pack, stream);
}
