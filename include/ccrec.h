/*
 * ccrec.h — C ABI of libccrec_hip.so, the MI355X (gfx950) hot path of the CubeCobra
 * denoising-autoencoder recommender.
 *
 * The reference has no FFI: its hot path sits behind Keras/TF Python objects
 * (SURVEY.md §8(b)).  Each entry point below names the reference code it replaces.
 * The Python host package (cubecobrarecommender_amd) binds these with ctypes; see
 * INTEGRATION.md for the binding a maintainer would add on the reference side.
 *
 * Conventions
 *   - All tensors are caller-owned DEVICE pointers (the library allocates nothing on
 *     the device except what a cc_trainer/cc_recommender is handed in its workspace).
 *   - Every call is stream-ordered on the given hipStream_t (passed as void*; NULL =
 *     default stream) and does not synchronise.
 *   - Return 0 on success, a negative CC_ERR_* code otherwise; no exceptions or aborts
 *     cross the ABI.  cc_last_error_string() gives the calling thread's last message.
 *   - Re-entrant: no global mutable state besides the thread-local error string.
 *   - Deterministic: given (seed, step) every kernel produces bit-identical outputs
 *     run to run (fixed-order reductions; the one float atomic — cc_gemm_mx8_bce_q's bias
 *     gradient over two 256-row tiles — adds two partials onto zero, which commutes).
 */
#ifndef CCREC_H
#define CCREC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CC_ABI_VERSION 2   /* 2: cc_tower_args gained y_bits, y_img, y_V */

enum cc_status {
  CC_OK = 0,
  CC_ERR_ARG = -1,         /* invalid argument / shape */
  CC_ERR_HIP = -2,         /* a HIP runtime call failed */
  CC_ERR_UNSUPPORTED = -3, /* shape or dtype this build does not handle */
  CC_ERR_CAPACITY = -4     /* a caller-provided buffer is too small */
};

/* CC_MX8: OCP MX-FP8 operands (cc_gemm only) — e4m3fn codes [rows][ld] + one E8M0 scale byte per
 * 32 K-elements ([rows][ld/32]), quantised by cc_quant_mx8 (config 5). */
enum cc_dtype { CC_F32 = 0, CC_BF16 = 1, CC_MX8 = 2 };

/* Number of tensors in the model (model.py: encoder 4 layers + 2 decoders x 4 layers, kernel+bias). */
#define CC_NUM_TENSORS 24

int cc_abi_version(void);
const char *cc_last_error_string(void);
/* Source identity: the first 32 hex digits of a SHA-256 over csrc/ + include/ (buildid.py),
 * compiled in by build.py.  Callers compare it with their tree to refuse a stale binary. */
const char *cc_build_id(void);

/* Host utility: CRC32C (Castagnoli) of [data, data+n) continuing from crc (0 to start) — the
 * checksum of TF tensor-bundle checkpoints (ml_files/<name>/variables). */
uint32_t cc_crc32c(uint32_t crc, const void *data, size_t n);

/* ----------------------------------------------------------------------------------
 * Parameter layout.  All weights live in ONE flat fp32 buffer (Adam m/v and the bf16
 * shadow use the same offsets).  Tensor order = Keras creation order (model.py:27-33,
 * 58-64, 92-98): encoder e1,e2,e3,bottleneck; decoder d1,d2,d3,reconstruct;
 * decoder_for_reg d1,d2,d3,reconstruct; each as (kernel [in,out] row-major, bias [out]).
 * offsets/sizes receive CC_NUM_TENSORS entries (elements); *total gets the flat size.
 * *main_total = elements of the encoder + decoder (D1) part, which comes first.
 * ---------------------------------------------------------------------------------- */
int cc_param_layout(int32_t V, int32_t d, int64_t *offsets, int64_t *sizes,
                    int64_t *total, int64_t *main_total);

/* ----------------------------------------------------------------------------------
 * F: noise + regulariser-row sampling.  Replaces DataGenerator.__getitem__ /
 * generate_data (src/ml/generator.py:38-103) — the law is restated in
 * oracle/noise_ref.py::philox_noise_batch (bit-exact).
 * ---------------------------------------------------------------------------------- */
typedef struct cc_noise_args {
  int32_t V;             /* cards */
  int32_t B;             /* cubes in this rank's batch */
  int32_t x_cap;         /* per-row capacity of x_idx (>= max cube size * 1.8) */
  int32_t with_reg;      /* 1: also draw one reg row per cube slot (rows B..2B-1 of x); 0: none
                            here — cc_reg_rows (owner computes) or the static full-mode identity
                            rows fill rows B.. of x */
  uint64_t seed;
  uint32_t slot_base;    /* rank * B: decorrelates ranks */
  int32_t batch_stride;  /* cubes consumed per global batch (B * world) */
  int32_t batch_offset;  /* rank * B */
  int32_t num_perms;     /* epochs cycle through num_perms permutations */
  int32_t num_cubes;     /* C */
  double noise_mean, noise_std;              /* generator.py:13-14 */
  const int64_t *cube_ptr;                   /* [C+1] CSR of the dataset */
  const int32_t *cube_idx;                   /* [nnz] sorted card ids per cube */
  const int32_t *perm;                       /* [num_perms, C] epoch permutations (generator.py:63-66) */
  const double *cdf;                         /* [V] normalised cumsum of neg_sampler */
  const double *neg_sampler;                 /* [V] generator.py:30 */
  const int32_t *guide;                      /* optional [2^guide_log2 + 1]: guide[g] =
                                                searchsorted_right(cdf, g / 2^guide_log2) */
  int32_t guide_log2;                        /* 0 = no guide table (full binary search) */
  const int64_t *state;                      /* device {step, batch_in_epoch, epoch, 0} */
  int32_t *x_cnt;                            /* [R] R = B (+ reg rows) */
  int32_t *x_idx;                            /* [R, x_cap] sorted card ids of x */
  uint32_t *y_bits;                          /* [B, ceil(V/32)] target bitmask */
  uint32_t *xt_bits;                         /* [V, ceil(R/32)] transposed x bits (zeroed) or NULL */
  int32_t *reg_idx;                          /* [B] (with_reg), [reg_cap] (cc_reg_rows) or NULL */
  int32_t *status;                           /* [1] device error flags (0 = ok) */
  int32_t xt_rows;                           /* rows of the E1 gradient product: xt_bits is
                                                [V, ceil(xt_rows/32)] (B, 2B, or B + reg_cap) */
  /* cc_reg_rows only (data parallel, M~ row-sharded, owner computes — SURVEY 8(e)): */
  int32_t reg_slots;                         /* global reg draws per step (B * world), slots 0.. */
  int32_t reg_lo, reg_hi;                    /* this rank's M~ rows [reg_lo, reg_hi) */
  int32_t reg_cap;                           /* reg rows of this rank: rows B..B+reg_cap-1 of x */
  uint32_t *x_bits;                          /* [rows, ceil(V/32)] x rows as bitmasks (rows F
                                                draws: B, or 2B with_reg), or NULL */
} cc_noise_args;
int cc_noise_fwd(const cc_noise_args *a, void *stream);
/* Owner-computes regulariser rows: draws the reg_slots global reg rows of the step
 * (slot s: the same Philox draw a one-process run of batch reg_slots makes for its slot s,
 * generator.py:47-51), keeps those whose card lies in [reg_lo, reg_hi) in slot order as rows
 * B, B+1, .. of x (x_cnt 1, reg_idx = card, xt bit set) and pads the rest of the reg_cap rows with
 * x_cnt 0 and reg_idx -1 (masked: no KL term, no gradient).  More than reg_cap owned draws set
 * status bit 2 (the surplus rows are dropped; reg_cap is sized ~6 sigma above the mean).
 * One 1024-thread workgroup; reads the step from state like cc_noise_fwd. */
int cc_reg_rows(const cc_noise_args *a, void *stream);
/* cc_adam_dense(p, m, v, g, shadow, n, next->state, ...) and, in the same launch, cc_noise_fwd
 * for the step AFTER next->state (step + 1, batch advanced with epoch roll-over as
 * cc_state_advance(batches_per_epoch) would) — the batch buffers must be free (this step's
 * backward done).  The state itself is not modified. */
int cc_adam_noise(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t n,
                  float lr, float beta1, float beta2, float eps, const cc_noise_args *next,
                  int64_t batches_per_epoch, void *stream);
/* cc_noise_fwd for the step AFTER a->state (the F half of cc_adam_noise alone): the data-parallel
 * step issues it beside its last gradient buckets' exchange (zero.py), so the next step's forward
 * starts without F.  Replaces the next __getitem__ (generator.py:38-103) the Keras fit loop makes
 * (train.py:99-102).  The state itself is not modified. */
int cc_noise_next(const cc_noise_args *a, int64_t batches_per_epoch, void *stream);
/* cc_adam_noise that also writes the updated bf16 values of the tower kernels into their
 * fragment-packed images (cc_tower_args.wpf / wpb order), so no cc_tower_transpose launch is
 * needed before the next forward (the step counters are then advanced by
 * cc_embed_gather_fwd_warm's state argument).  pack->off[l] is the element offset of layer l's
 * [K][N] kernel in the flat buffers. */
typedef struct cc_adam_pack {
  int32_t n;             /* layers (<= 9) */
  int32_t K[9], N[9];
  int64_t off[9];
  void *wpf[9];
  void *wpb[9];
} cc_adam_pack;
int cc_adam_noise_pack(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t n,
                       float lr, float beta1, float beta2, float eps, const cc_noise_args *next,
                       int64_t batches_per_epoch, const cc_adam_pack *pack, void *stream);
/* cc_adam_noise_pack over the two flat ranges [lo0, lo0 + n0) and [lo1, lo1 + n1) of the buffers at
 * p, m, v, g, shadow (lo1 >= lo0 + n0; n1 may be 0; range starts multiples of 4); pack->off[l]
 * counts from p and every packed layer lies inside one of the ranges. */
int cc_adam_noise_pack2(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t lo0,
                        int64_t n0, int64_t lo1, int64_t n1, float lr, float beta1, float beta2, float eps,
                        const cc_noise_args *next, int64_t batches_per_epoch, const cc_adam_pack *pack,
                        void *stream);
/* cc_adam_noise_pack2 without F (the next step's F drawn by cc_tower_bwd_chain_noise); `next` is
 * checked as there but not drawn. */
int cc_adam_pack2(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t lo0, int64_t n0,
                  int64_t lo1, int64_t n1, float lr, float beta1, float beta2, float eps,
                  const cc_noise_args *next, int64_t batches_per_epoch, const cc_adam_pack *pack, void *stream);

/* ----------------------------------------------------------------------------------
 * E1 forward: H[r] = ReLU(sum_{j in x_r} W1[j] + b1).  Replaces Dense(d)(x) on the 0/1
 * cube (model.py:27,36): a coalesced row gather instead of a dense [R,V]x[V,d] GEMM.
 * table is bf16 (CC_BF16) or fp32 (CC_F32) [V, d]; out is the same dtype [R, d].
 * ---------------------------------------------------------------------------------- */
int cc_embed_gather_fwd(int32_t dtype, const void *table, const float *bias, int32_t V,
                        int32_t d, int32_t R, const int32_t *x_cnt, const int32_t *x_idx,
                        int32_t x_cap, void *out, void *stream);
/* cc_embed_gather_fwd + the L2 warm-up of cc_splitk_reduce_warm for the next launch (the tower
 * forward's packed weights; bf16 d = 256 only, other shapes ignore it) and, with state non-NULL,
 * the previous step's cc_state_advance(batches_per_epoch) (nothing in a step reads the counters
 * before its Adam launch). */
int cc_embed_gather_fwd_warm(int32_t dtype, const void *table, const float *bias, int32_t V, int32_t d,
                             int32_t R, const int32_t *x_cnt, const int32_t *x_idx, int32_t x_cap,
                             void *out, const void *warm, int64_t warm_bytes, int64_t *state,
                             int64_t batches_per_epoch, void *stream);
/* cc_embed_gather_fwd_warm that, with xt_bits non-NULL, also writes the whole W1-gradient
 * bitmask as the bit transpose of F's x row bitmasks (cc_noise_args.x_bits [R, ceil(V/32)]):
 * xt_bits[card * ceil(xt_rows/32) + row/32] bit row%32 = x_bits[row] bit card, rows < xt_rows,
 * every word written (no zeroed xt needed) — the bits cc_noise_fwd sets by atomics when its
 * xt_bits is non-NULL.  One process gives F x_bits instead of xt_bits: F's next-step draw runs
 * inside the HBM-bound Adam launch, where its scattered atomics queued behind the Adam streams;
 * here (bf16 d = 256) the transpose rides as extra blocks of the latency-bound gather. */
int cc_embed_gather_fwd_xt(int32_t dtype, const void *table, const float *bias, int32_t V, int32_t d,
                           int32_t R, const int32_t *x_cnt, const int32_t *x_idx, int32_t x_cap,
                           void *out, const void *warm, int64_t warm_bytes, int64_t *state,
                           int64_t batches_per_epoch, const uint32_t *x_bits, uint32_t *xt_bits,
                           int32_t xt_rows, void *stream);

/* ----------------------------------------------------------------------------------
 * E1 backward: dW1[r] = sum_{b : r in x_b} dpre[b] (ascending b, deterministic), for every
 * row r of W1 (dense, as TF's MatMul gradient is dense).  xt_bits [V, ceil(R/32)] is CONSUMED:
 * it is left all-zero, ready for the next step's cc_noise_fwd (which ORs bits into it).
 * Writes grad [V, d] fp32 and, when bias_grad != NULL, bias_grad[c] = sum_b dpre[b, c] (db1).
 * Replaces the MatMul/BiasAdd gradients of model.py:27 inside fit.
 * ---------------------------------------------------------------------------------- */
int cc_embed_scatter_bwd(const float *dpre, int32_t V, int32_t d, int32_t R,
                         const uint32_t *xt_bits, float *grad, float *bias_grad, void *stream);
/* The same gradient on bf16 MFMA (the bf16/fp8 training path): dW1 = X^T dPre1 with the x^T
 * bitmask expanded to 0/1 bf16 A fragments in registers and dpre_t = dPre1^T bf16 [d][ld_t]
 * (ld_t % 64 == 0 is the row stride; rows 0..R-1 enter the product, columns R..ceil64(R)-1 zero;
 * cc_tower_args.gpre1t).  d % 128 == 0, R <= 2048.
 * Consumes (zeroes) xt_bits like cc_embed_scatter_bwd; deterministic. */
int cc_embed_grad_mfma(const void *dpre_t, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                       uint32_t *xt_bits, float *grad, float *bias_grad, void *stream);
/* cc_embed_grad_mfma with B = dPre1 as packed transposed fragments (cc_tower_args.gpre1p,
 * reduction stride ld_t >= ceil64(R); the first R rows enter the product): each wave streams its 64 columns' fragments straight from
 * L2 (1 KB per wave load), no LDS staging or per-K-tile barriers.  d == 256. */
int cc_embed_grad_packed(const void *dpre_p, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                         uint32_t *xt_bits, float *grad, float *bias_grad, void *stream);
/* The same gradient by column slice (the training path's default): one workgroup per (32-row
 * chunk of W1 rows, 32 columns) stages its dPre1 slice and bit words in LDS once.  dpre is the
 * packed transposed image (packed != 0, cc_tower_args.gpre1p) or dPre1^T [d][ld_t] (packed == 0,
 * cc_tower_args.gpre1t); d % 32 == 0, R <= 2048.  tickets: cc_embed_grad_cs_tickets(V, d, R)
 * uint32 words, zero before the first call and left zero by every call (the last workgroup of a
 * chunk to stage its bit words clears them in xt_bits and resets its ticket); tickets NULL leaves
 * xt_bits as it is (for callers that rewrite every word, cc_embed_gather_fwd_xt).  Bit-identical to
 * cc_embed_grad_mfma / cc_embed_grad_packed (same MFMA k order); consumes xt_bits likewise. */
int cc_embed_grad_cs(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                     uint32_t *xt_bits, float *grad, float *bias_grad, uint32_t *tickets, void *stream);
int32_t cc_embed_grad_cs_tickets(int32_t V, int32_t d, int32_t R);
/* cc_embed_grad_cs with TF Adam (cc_adam_dense's update, t = state[0] + 1) applied to W1 in the
 * kernel's epilogue (one process: the gradient is final there): p, m, v are W1's rows [V][d] of
 * the flat fp32 buffers, shadow its bf16 rows; the W1 gradient itself is never stored, the bias
 * gradient goes to bias_grad for the main Adam launch (which then starts after W1).  Bit-identical
 * parameters / moments to cc_embed_grad_cs followed by cc_adam_dense over W1. */
int cc_embed_grad_cs_adam(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                          uint32_t *xt_bits, float *bias_grad, uint32_t *tickets, float *p, float *m, float *v,
                          uint16_t *shadow, const int64_t *state, float lr, float beta1, float beta2, float eps,
                          void *stream);
/* The same two products with the sampled regulariser's identity rows taken by index (reference:
 * generator.py:47-61, x_reg = the identity rows of the reg draws; train.py:99-102 fits on them): the
 * bit matrix holds the first R (cube) rows only and the dPre1 image holds the nreg reg rows as its
 * rows 16 reg_k0 .. (reg_k0 >= R / 16), row 16 reg_k0 + i being the one-card row {reg_idx[i]}
 * (reg_idx[i] < 0: a padding row, in the bias row's sum only).  Each 32-row tile adds the reg
 * k-steps whose A fragment is not all zero for it (every one for the bias row), ascending, after
 * the cube k-steps: bit-identical to the same products over R + nreg rows with the reg rows' bits in
 * xt_bits.  nreg <= 512; card0: the card of W1 row 0 (a row chunk's first row; 0 for the Adam form). */
int cc_embed_grad_cs_reg(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                         uint32_t *xt_bits, float *grad, float *bias_grad, uint32_t *tickets,
                         const int32_t *reg_idx, int32_t nreg, int32_t reg_k0, int32_t card0, void *stream);
int cc_embed_grad_cs_adam_reg(const void *dpre, int32_t packed, int32_t V, int32_t d, int32_t R, int32_t ld_t,
                              uint32_t *xt_bits, float *bias_grad, uint32_t *tickets, float *p, float *m,
                              float *v, uint16_t *shadow, const int64_t *state, float lr, float beta1,
                              float beta2, float eps, const int32_t *reg_idx, int32_t nreg, int32_t reg_k0,
                              void *stream);
/* Full-mode regulariser (all |V| one-hot identity rows, README.md:27 KL(M, D2(E(I)))): the rows'
 * W1 gradient is dPre1 itself — grad[lo + r] += round(dpre[r]) for r < n and, with bias_grad,
 * bias_grad += sum_r round(dpre[r]) in a fixed order; round = bf16 RNE for dtype CC_BF16 (the
 * operand rounding of the MFMA path), none for CC_F32.  Run after the cube rows' E1 gradient.
 * partial: cc_embed_identity_ws(n, d) bytes of scratch. */
size_t cc_embed_identity_ws(int32_t n, int32_t d);
int cc_embed_identity_add(int32_t dtype, const float *dpre, int32_t n, int32_t d, int32_t lo,
                          float *grad, float *bias_grad, float *partial, void *stream);

/* ----------------------------------------------------------------------------------
 * Generic MFMA GEMM with fused epilogues — the Dense layers of the E/D towers and the
 * decoder output layers (model.py:29-33, 58-64).  C[M,N] = op(A)[M,K] op(B)[K,N].
 *   ta: A stored [K, M] (else [M, K]);  tb: B stored [N, K] (else [K, N]).  Row-major.
 *   dtype: operand dtype (CC_BF16 -> v_mfma_f32_32x32x16_bf16, CC_F32 -> v_mfma_f32_32x32x2_f32);
 *   accumulation always fp32.
 * ---------------------------------------------------------------------------------- */
enum cc_epilogue {
  CC_EPI_STORE = 0,     /* out = act(acc + bias) -> C (dtype) and/or Cf (fp32) */
  CC_EPI_BCE = 1,       /* D1 logits -> BCE loss partials + dZ (train.py:85) */
  CC_EPI_MASK = 2,      /* out = acc * (H[m,n] > 0) -> C (dtype) and/or Cf: ReLU backward */
  CC_EPI_SPLITK = 3     /* raw fp32 partial per K split -> Cf + split*M*N */
};
typedef struct cc_gemm_args {
  int32_t dtype, ta, tb, epilogue;
  int32_t M, N, K, lda, ldb, ldc;
  int32_t splits;       /* K splits (CC_EPI_SPLITK only) */
  int32_t relu;         /* CC_EPI_STORE */
  const void *A, *B;
  const float *bias;    /* [N] or NULL */
  void *C;              /* dtype output or NULL */
  float *Cf;            /* fp32 output or NULL */
  const void *H;        /* CC_EPI_MASK: [M, ldc] dtype activations whose sign gates the gradient */
  const uint32_t *y_bits; /* CC_EPI_BCE: [M, ceil(N/32)] targets */
  float scale;          /* CC_EPI_BCE: 1/(B*V) */
  double *loss_partials;  /* CC_EPI_BCE: [gridDim.x*gridDim.y] */
  float *colsum;        /* optional [N] ([splits, N] with CC_EPI_SPLITK): colsum[n] = sum_k op(B)[k, n]
                           (fp32, ascending k) — the bias gradient of a Dense layer fused into its
                           dW = X^T dPre product */
  void *Ct;             /* CC_EPI_BCE, optional: dZ^T [N][ldct] (dtype) — the k-contiguous operand of
                           dW = H^T dZ, written with packed stores from the accumulator registers */
  int32_t ldct;
  double *loss_out;     /* CC_EPI_BCE, optional: loss_out[0] = sum(loss_partials) * loss_scale, in
                           tile order (the same as cc_reduce_loss would give), computed by the
                           kernel's last tile block */
  double loss_scale;
  uint32_t *ticket;     /* with loss_out: one zeroed word, left zeroed */
  const uint8_t *a_scale, *b_scale;  /* CC_MX8: E8M0 scales [M][lda/32] of A, [N][ldb/32] of B */
} cc_gemm_args;
int cc_gemm(const cc_gemm_args *g, void *stream);
/* cc_gemm with the MX-FP8 products kept on the 128 x 128 register-staged kernel instead of the
 * 256 x 256 LDS-DMA one (identical MFMA order per output): the reference side of the bit-identity
 * tests (tests/test_gpu_mx8.py); other dtypes behave as cc_gemm. */
int cc_gemm_tile128(const cc_gemm_args *g, void *stream);
/* CC_MX8 runs v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3, block scales applied in the MFMA):
 * NT only (ta = 0, tb = 1), K % 128 == 0, lda % 128 == ldb % 128 == 0, epilogues STORE / BCE /
 * SPLITK without colsum; outputs as for CC_BF16 (C is bf16, Cf fp32). */
/* Two independent products in one launch (grouped GEMM) when both take the bf16 NT path with
 * the STORE or SPLITK epilogue; otherwise cc_gemm(g0) then cc_gemm(g1).  Same results. */
int cc_gemm_pair(const cc_gemm_args *g0, const cc_gemm_args *g1, void *stream);
/* MX-FP8 NT product(s) on 256 x 256 tiles with an LDS-DMA pipeline (mx8gemm.hip): epilogue STORE
 * (optional bias, fp32 Cf and/or bf16 C) or SPLITK; g1 optional (a second problem in the same
 * launch).  cc_gemm / cc_gemm_pair route their MX8 STORE / SPLITK calls here; bit-identical to the
 * 128 x 128 MX kernel.  Needs K, lda, ldb multiples of 128 and operands below 2 GB. */
int cc_gemm_mx8_wide(const cc_gemm_args *g0, const cc_gemm_args *g1, void *stream);
/* Config 5's decoder output layer (model.py:64,94; train.py:85) on the 256 x 256 MX-FP8 kernel with
 * the dZ operand images made in the BCE epilogue: zq [M][ldzq] + zqs (K = N, for dX), ztq [N][ldztq]
 * + ztqs (K = M, for dW) bit-exact with cc_quant_mx8 of the bf16 dZ / dZ^T, and colsum[N] = the bias
 * gradient (zeroed here).  g->C / g->Ct (bf16 dZ / dZ^T) optional.  M % 32 == 0, M <= 512. */
int cc_gemm_mx8_bce_q(const cc_gemm_args *g, uint8_t *zq, int32_t ldzq, uint8_t *zqs, uint8_t *ztq,
                      int32_t ldztq, uint8_t *ztqs, float *colsum, void *stream);
/* cc_gemm_mx8_bce_q + an independent MX8 STORE / SPLITK product g2 (config 5: the regulariser
 * branch's logits) as extra blocks of the same launch; g2 = NULL is cc_gemm_mx8_bce_q. */
int cc_gemm_mx8_bce_q2(const cc_gemm_args *g, uint8_t *zq, int32_t ldzq, uint8_t *zqs, uint8_t *ztq,
                       int32_t ldztq, uint8_t *ztqs, float *colsum, const cc_gemm_args *g2, void *stream);
/* workspace bound for cc_gemm's loss partials: ceil(M/64)*ceil(N/64) doubles */
int cc_gemm_grid(int32_t M, int32_t N, int32_t *tiles);

/* Sum K-split partials (in split order) and apply the MASK/STORE epilogue; when colsum_out is
 * given, also colsum_out[n] = sum_z colsum_partials[z*N + n] (cc_gemm's split-K colsum rows). */
int cc_splitk_reduce(int32_t dtype, const float *partials, int32_t splits, int32_t M, int32_t N,
                     const void *H, void *C, float *Cf, const float *colsum_partials,
                     float *colsum_out, void *stream);
/* ... and, at the end of every workgroup, one dword per 128-B line of [warm, warm + warm_bytes)
 * read by the workgroups of each XCD in turn: the next launch (the tower backward's packed
 * weights) finds them in every XCD's L2.  Results identical to cc_splitk_reduce. */
int cc_splitk_reduce_warm(int32_t dtype, const float *partials, int32_t splits, int32_t M, int32_t N,
                          const void *H, void *C, float *Cf, const float *colsum_partials,
                          float *colsum_out, const void *warm, int64_t warm_bytes, void *stream);

/* MX-FP8 quantisation (oracle/mx8_ref.py, bit-exact): blocks of 32 along the GEMM K axis, E8M0
 * exponent e = min{e : amax <= 448 * 2^e}, codes = e4m3 RNE of x * 2^-e.  src is [rows][ld_src]
 * (dtype CC_BF16 or CC_F32).
 *   transpose = 0: dst [rows][ld_dst] codes, scales [rows][ld_dst/32]; K axis = cols (padded with
 *                  zeros up to ld_dst); rowsum (optional, needs ld_dst <= 2048): rowsum[r] = fp32
 *                  sum of src row r (the bias gradient when src is dZ^T).
 *   transpose = 1: dst [cols][ld_dst] with dst[c][r] = q(src[r][c]), scales [cols][ld_dst/32];
 *                  K axis = rows (padded up to ld_dst).  rowsum must be NULL.
 * ld_dst % 128 == 0. */
int cc_quant_mx8(int32_t dtype, const void *src, int32_t rows, int32_t cols, int32_t ld_src,
                 int32_t transpose, uint8_t *dst, int32_t ld_dst, uint8_t *scales, float *rowsum,
                 void *stream);
/* Both MX-FP8 images of src [rows][cols] from one read: dst_t [cols][ld_t] + scales_t (K = rows, =
 * cc_quant_mx8 transpose=1) and dst_r [rows][ld_r] + scales_r (K = cols, = transpose=0), each
 * bit-exact with cc_quant_mx8.  Config 5's decoder output kernels after every Adam step. */
int cc_quant_mx8_both(int32_t dtype, const void *src, int32_t rows, int32_t cols, int32_t ld_src,
                      uint8_t *dst_t, int32_t ld_t, uint8_t *scales_t, uint8_t *dst_r, int32_t ld_r,
                      uint8_t *scales_r, void *stream);

/* dst[c][r] = src[r][c] for a [rows, cols] row-major matrix (dtype elements). */
int cc_transpose(int32_t dtype, const void *src, int32_t rows, int32_t cols, void *dst, void *stream);

/* out[n] (+)= sum_r X[r, n] (fp32 accumulate, ascending r). db of every Dense layer. */
int cc_colsum(int32_t dtype, const void *X, int32_t R, int32_t N, int32_t ld, float *out,
              void *stream);

/* ----------------------------------------------------------------------------------
 * Fused towers (model.py:29-33 E2..E4, :58-62 D1..D3 of both decoders) on 32-row blocks.
 * Rows [0,B) use `decoder`, rows [B,R) `decoder_for_reg`; one block never straddles B.
 * Layer order l = 0..8: e2, e3, e4 | d1, d2, d3 (decoder) | d1, d2, d3 (decoder_for_reg).
 *   cc_tower_fwd: act[0] = H1 (input) -> act[1..6] = H2, H3, Zl, D1, D2, D3 (bias+ReLU fused).
 *   cc_tower_bwd: from gD3 = dPre of d3 [R,d] down to gpre1 = dPre of e1 [R,d] fp32 (the dX
 *                 chain, writing every layer's dPre to gact), then the per-(layer, 32-row block)
 *                 partial dW/db of the 6 layers each block touches into slab[blk][...].
 *   cc_tower_reduce: grads of the 9 layers = sum of the slabs in block order (deterministic).
 *   cc_tower_transpose: wt[l] = w[l]^T ([N][K]) — the k-contiguous operand the forward reads.
 * d <= 1024 (bf16) / <= 256 (fp32); the generic cc_gemm path covers larger widths.
 * ---------------------------------------------------------------------------------- */
typedef struct cc_tower_args {
  int32_t dtype, d, B, R;
  const void *w[9];      /* [K][N] dtype */
  void *wt[9];           /* [N][K] dtype */
  const float *b[9];     /* [N] */
  void *act[7];          /* H1, H2, H3, Zl, D1, D2, D3: [R, width] dtype */
  void *act6t;           /* optional: D3^T [d][R] dtype (k-contiguous operand of the decoder dW) */
  const void *gD3;       /* [R, d] dtype */
  void *gact[5];         /* bwd outputs, dPre of e2, e3, e4, d1, d2: [R, N_l] dtype */
  float *gpre1;          /* [R, d] fp32 */
  float *slab;           /* [R/32, cc_tower_slab_elems(d)] fp32 */
  float *gw[9];          /* reduce outputs: kernel grads [K][N] */
  float *gb[9];          /* bias grads [N] */
  void *gpre1t;          /* optional (bf16): dPre1^T [d][ceil64(R)] for cc_embed_grad_mfma */
  /* optional (bf16, d <= 256): MFMA-fragment-packed weight images, K*N elements each, written by
   * cc_tower_transpose.  Fragment (t, j) of a [rows][red] operand = 64 lanes x 8 consecutive
   * elements, lane l holding row 32t + (l & 31), reduction 16j + 8(l >> 5) .. +8, stored as one
   * contiguous 1 KB run: every wave load reads whole cache lines.
   *   wpf: forward B operand (rows = N outputs, reduction K): element W[k][n];
   *   wpb: backward B operand (rows = K outputs, reduction N): element W[k][n].
   * Used by the fast tower kernels when all of them are set. */
  void *wpf[9];
  void *wpb[9];
  /* optional (bf16, the fast d <= 256 and wide d <= 1024 kernels): D3 as fragment-packed MFMA
   * operand images for cc_dec_bce_dw / cc_dec_softmax_kl_dw — act6p: rows = batch rows, reduction d ([R/32][d/16][64][8]); act6tp: rows = d,
   * reduction = batch rows ([d/32][R/16][64][8]).  Same fragment order as wpf. */
  void *act6p;
  void *act6tp;
  /* optional (bf16, d <= 256, fast kernels; all twelve set): packed transposed images of every
   * layer's input H_i [R][K_i] (written by cc_tower_fwd) and output gradient G_i [R][N_i]
   * (cc_tower_bwd_chain), rows = features, reduction = batch rows, act6tp's layout; with them
   * cc_tower_bwd_dw_direct runs one MFMA chain per 32x32 dW tile straight from these images. */
  void *hpt[6];
  void *gpt[6];
  /* optional (bf16, d <= 256): dPre1 [R][d] as packed transposed fragments with reduction length
   * ceil64(R) (rows past R stay zero: allocate zeroed) — cc_embed_grad_packed's B operand; when
   * set, the fast backward chain writes it instead of gpre1t. */
  void *gpre1p;
  /* optional (bf16, d <= 256): cc_tower_fwd also writes the W1-gradient bitmask xt_bits
   * [xt_V][ceil(xt_rows/32)] as the bit transpose of x_bits [>= xt_rows][ceil(xt_V/32)] (as
   * cc_embed_gather_fwd_xt does), in extra blocks beside the 32-row tower chains (NULL: no). */
  const void *x_bits;
  void *xt_bits;
  int32_t xt_V, xt_rows;
  /* optional (config 5: bf16 towers with MX-FP8 decoder GEMMs, 256 < d, the wide chains): cc_tower_fwd
   * also writes D3's MX-FP8 operand images exactly as cc_quant_mx8 would from D3 — d3q [R][d] codes
   * with d3qs [R][d/32] E8M0 scales (K = d), d3tq [d][R] with d3tqs [d][R/32] (K = batch rows) —
   * from the LDS copy it already holds (all four set, or none). */
  void *d3q, *d3qs, *d3tq, *d3tqs;
  /* optional (bf16 fast chains, d <= 256): cc_tower_fwd also writes y_img [ceil(y_V/32)][B] uint32,
   * the target row bitmasks y_bits [B][ceil(y_V/32)] transposed for the fused D1 kernel's lane masks
   * (cc_dec_bce_dw_img): word column w, then the B rows with every 32-row block in accumulator-
   * register order — dword 2r + h of a block = its row (r & 3) + 8 (r >> 2) + 4h — in extra blocks
   * beside the chains (NULL: no). */
  const void *y_bits;
  void *y_img;
  int32_t y_V;
} cc_tower_args;
int64_t cc_tower_slab_elems(int32_t d);
int cc_tower_fwd(const cc_tower_args *t, void *stream);
int cc_tower_bwd(const cc_tower_args *t, void *stream);
/* cc_tower_bwd = cc_tower_bwd_chain (dX chain; writes gpre1 and every layer's dPre) followed by
 * cc_tower_bwd_dw (per-block dW/db slabs); split so the slabs can overlap the E1 scatter. */
int cc_tower_bwd_chain(const cc_tower_args *t, void *stream);
/* cc_tower_bwd_chain plus, in extra workgroups of the same launch (on the CUs the 32-row chains
 * leave idle), exactly cc_adam_dense over the flat ranges [lo0, lo0 + n0) and [lo1, lo1 + n1) of
 * p, m, v, g, shadow (lo1 >= lo0 + n0, n1 may be 0, starts multiples of 4) — ranges the chains do
 * not read (the trainer: trailing parts of the decoder output layers, whose gradients are final
 * after the output-layer kernels and whose bf16 shadows the dX products have already consumed).
 * bf16 fast chains (d <= 256) only. */
int cc_tower_bwd_chain_adam(const cc_tower_args *t, float *p, float *m, float *v, const float *g,
                            uint16_t *shadow, int64_t lo0, int64_t n0, int64_t lo1, int64_t n1,
                            const int64_t *state, float lr, float beta1, float beta2, float eps, void *stream);
/* cc_tower_bwd_chain plus F of the NEXT step (generator.py:38-103, exactly cc_noise_fwd's draws for
 * the state {step + 1, batch + 1 (epoch rollover at batches_per_epoch), epoch}, as the Adam + F
 * launch draws them) in extra workgroups, two cubes each, and — when n0 + n1 > 0 — TF Adam over two
 * flat ranges as cc_tower_bwd_chain_adam.  F writes x / y / reg rows but no xt bits (next->xt_bits
 * must be NULL: the W1 gradient after this launch still reads them); every batch buffer it writes
 * has been read for this step by the tower backward.  bf16 fast chains (d <= 256) only. */
int cc_tower_bwd_chain_noise(const cc_tower_args *t, const cc_noise_args *next, int64_t batches_per_epoch,
                             float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t lo0,
                             int64_t n0, int64_t lo1, int64_t n1, const int64_t *state, float lr, float beta1,
                             float beta2, float eps, void *stream);
int cc_tower_bwd_dw(const cc_tower_args *t, void *stream);
int cc_tower_reduce(const cc_tower_args *t, void *stream);
/* bf16: every layer's dW/db written directly (no slabs, no reduce): cc_tower_bwd_dw +
 * cc_tower_reduce in one launch; row-order MFMA sums, deterministic. */
int cc_tower_bwd_dw_direct(const cc_tower_args *t, void *stream);
int cc_tower_transpose(const cc_tower_args *t, void *stream);
/* cc_tower_transpose + cc_state_advance(state, batches_per_epoch) in the same launch */
int cc_tower_transpose_advance(const cc_tower_args *t, int64_t *state, int64_t batches_per_epoch,
                               void *stream);

/* ----------------------------------------------------------------------------------
 * D1 output layer fused with sigmoid+BCE (model.py:64,94; train.py:85): logits
 * z = H3 Wo + bo are never written; dZ = (sigmoid(z) - y)/(B*V) is.
 * D2 softmax + KL (model.py:98; train.py:85): per reg row, row-softmax of z2, KL against the
 * M~ row, dZ2 = reg/B * p (g - <p,g>) with the clip semantics of SURVEY §8(a) A9.
 * ---------------------------------------------------------------------------------- */
int cc_dec_bce_fused(int32_t dtype, const void *H3, const void *Wo, const float *bo,
                     int32_t B, int32_t d, int32_t V, const uint32_t *y_bits, void *dZ,
                     double *loss_partials, int32_t *n_partials, void *stream);
/* D1 output layer in one pass (bf16; B in {128, 256, 512}, d in {128, 256, 512}): per
 * 96-column (d = 512: 64-column) slice of V, logits z = D3 Wo + bo (Wo as Wo^T [V][d]; with WoT NULL the [d][V] weights Wo
 * themselves, each block transposing its slice in LDS — no Wo^T copy to refresh after Adam;
 * D3p / D3tp: optional packed operand images, cc_tower_args.act6p / act6tp), dZ = (sigmoid(z) - y)/(B*V) written
 * row-major [B][V] (for the dX product), and dWo [d][V] = D3^T dZ (D3t = D3^T [d][ldt]) and
 * dbo = colsum dZ from the block's LDS copy of dZ^T — no dZ^T in HBM, no separate dW launch.
 * loss_partials: cc_dec_bce_dw_blocks(V) doubles; loss_out (optional, with ticket) =
 * sum(partials) * loss_scale reduced by the last block. */
int cc_dec_bce_dw(const void *D3, const void *D3t, int32_t ldt, const void *D3p, const void *D3tp,
                  const void *WoT, const void *Wo, const float *bo,
                  int32_t B, int32_t d, int32_t V, const uint32_t *y_bits, void *dZ, float *gW,
                  float *gb, double *loss_partials, double *loss_out, double loss_scale,
                  uint32_t *ticket, void *stream);
/* cc_dec_bce_dw with dZ's row pitch ldz (>= V; a multiple of 64 keeps every dZ row 128-B aligned, so
 * no cache line of dZ is written in parts by two output slices or two rows: no partial-line
 * read-modify-write). */
int cc_dec_bce_dw_ld(const void *D3, const void *D3t, int32_t ldt, const void *D3p, const void *D3tp,
                     const void *WoT, const void *Wo, const float *bo, int32_t B, int32_t d, int32_t V,
                     const uint32_t *y_bits, void *dZ, int32_t ldz, float *gW, float *gb, double *loss_partials,
                     double *loss_out, double loss_scale, uint32_t *ticket, void *stream);
/* cc_dec_bce_dw_ld with the targets also as y_img (cc_tower_args.y_img, 128-B aligned, written from
 * this y_bits by the tower forward launch): the epilogue's lane masks then come in two scalar 64-B
 * loads per 32-column tile instead of 32 scattered word loads.  Same results, bit for bit. */
int cc_dec_bce_dw_img(const void *D3, const void *D3t, int32_t ldt, const void *D3p, const void *D3tp,
                      const void *WoT, const void *Wo, const float *bo, int32_t B, int32_t d, int32_t V,
                      const uint32_t *y_bits, const uint32_t *y_img, void *dZ, int32_t ldz, float *gW, float *gb,
                      double *loss_partials, double *loss_out, double loss_scale, uint32_t *ticket, void *stream);
int32_t cc_dec_bce_dw_blocks(int32_t V);
/* D2 softmax + KL on materialised fp32 logits Z2 [B][V] (model.py:98, train.py:85, TF 2.5 clip
 * semantics): row b uses the M~ row y_reg + reg_idx[b] * V; dZ[b] = scale * ([p >= 1e-7](-t) +
 * p * sum_{p>=1e-7} t) with scale = reg * (the row's weight in the objective, e.g. 1/B);
 * kl_partials[b] = KL of row b.  reg_idx[b] < 0 marks a padding row: dZ[b] = 0, partial 0. */
int cc_dec_softmax_kl_fused(int32_t dtype, const float *Z2, int32_t B, int32_t V,
                            const float *y_reg, const int32_t *reg_idx, float scale, void *dZ,
                            double *kl_partials, void *stream);
/* cc_dec_softmax_kl_fused (bf16 dZ) also writing dZ's MX-FP8 row image zq [B][ldzq] + zqs (K = V,
 * bit-exact with cc_quant_mx8 of the bf16 dZ): config 5's regulariser branch. */
int cc_dec_softmax_kl_q(const float *Z2, int32_t B, int32_t V, const float *y_reg, const int32_t *reg_idx,
                        float scale, void *dZ, double *kl_partials, uint8_t *zq, int32_t ldzq, uint8_t *zqs,
                        void *stream);
/* D2 output layer fused (decreg.hip): logits -> softmax -> KL vs M~ rows -> dZ -> dWo/dbo with
 * no fp32 logits in HBM (model.py:64/98, train.py:85; TF 2.5 clip semantics).  Row r of the
 * regulariser rows is row row0 + r of the packed D3 images D3p ([R/32][d/16][64][8], act6p) and
 * D3tp ([d/32][ldt/16][64][8], act6tp); Wo [d][V] bf16 is read in place; Mt + card * V is the
 * M~ row of card reg_idx[r] (-1: padding row, contributes nothing); tsum[2 card], tsum[2 card + 1]
 * = sum_j t, sum_j t ln t over t = clip(M~[card, j], 1e-7, 1) (cc_kl_tsum), indexed like Mt.
 * Outputs: dZ [rows][V] bf16 (= scale * ([p >= 1e-7](-t) + p * sum_{p>=1e-7} t), for the dX
 * product), gW [d][V], gb [V], loss_partials (cc_dec_kl_blocks(V) doubles) and, with ticket,
 * loss_out = sum * loss_scale.  d in {128, 256, 512} (96-column slices, 64 at d = 512), rows % 32
 * == 0.  More than 512 rows (the full-mode regulariser) with V even: gW = D3^T dZ by a separate
 * launch over the stored dZ.  ws: cc_dec_kl_ws_size(rows, V) bytes, 16-B aligned. */
typedef struct cc_dec_kl_args {
  int32_t d, V, rows, ldt, row0;
  const void *D3p, *D3tp, *Wo;
  const float *bo, *Mt, *tsum;
  int64_t mt_bytes;          /* bytes of Mt addressable from its base (rows of the shard end at it) */
  int32_t mt_lo;             /* first card whose M~ row is resident (the shard's lo; 0 unsharded) */
  const int32_t *reg_idx;
  float scale;
  void *dZ;
  float *gW, *gb;
  double *loss_partials, *loss_out;
  double loss_scale;
  uint32_t *ticket;
  void *ws;
  int32_t flags;             /* 0, or CC_KL_DWO_NARROW: with many rows (full mode) dWo by the 96-column
                                kernel in one pass over all rows instead of kl_dwo2's two row halves
                                (the default at d = 256, |V| % 8 == 0; dWo differs by float rounding).
                                The round-5 A/B paths measured slower (M~ staged through LDS, M~ as
                                16-B rows, dWo by producer waves) were retired (branch archive/r05-ab-knobs). */
} cc_dec_kl_args;
#define CC_KL_DWO_NARROW 16
size_t cc_dec_kl_ws_size(int32_t rows, int32_t V);
int32_t cc_dec_kl_blocks(int32_t V);
int cc_dec_softmax_kl_dw(const cc_dec_kl_args *a, void *stream);
/* Row constants of the n rows of Mt (once per M~), t = clip(Mt[i * V + j], 1e-7, 1):
 * tsum[2i] = sum_j t, tsum[2i + 1] = sum_j t ln t (the KL's target-entropy part) */
int cc_kl_tsum(const float *Mt, int32_t n, int32_t V, float *tsum, void *stream);

/* ----------------------------------------------------------------------------------
 * Keras metrics=['accuracy'] of the two outputs (train.py:83-88; metrics.hip), counted on the device
 * (integer atomics: order-free totals).  Z: fp32 logits [rows][ldz].  TF 2.5 resolves 'accuracy' by
 * shape (compile_utils._get_metric_object: binary only for a last dim of 1), so both [B, V] outputs
 * report categorical_accuracy.
 * cc_sigmoid_cat_accuracy: count += #{r : argmax_j sigmoid(Z[r][j]) == first set bit of y row r (0 if
 *   none)} over B rows, sigmoid in fp32 saturating to 1 from z >= 15.7243833541870117 (Eigen's float
 *   logistic), first index on ties; y_bits [B][ceil(V/32)] as cc_dec_bce_dw's.
 * cc_row_argmax: out[r] = first index of the maximum of X[r][0..V) (tf.argmax).
 * cc_cat_accuracy: for the rows with reg_idx[r] >= 0: count[1] += 1 and count[0] += [argmax Z[r] ==
 *   t_argmax[reg_idx[r] - t_lo]] (categorical_accuracy of the softmax output vs the M~ row). */
int cc_sigmoid_cat_accuracy(const float *Z, int32_t ldz, const uint32_t *y_bits, int32_t B, int32_t V,
                            unsigned long long *count, void *stream);
int cc_row_argmax(const float *X, int64_t ld, int32_t rows, int32_t V, int32_t *out, void *stream);
int cc_cat_accuracy(const float *Z, int32_t ldz, int32_t rows, int32_t V, const int32_t *reg_idx,
                    const int32_t *t_argmax, int32_t t_lo, unsigned long long *count, void *stream);
/* Decoder dX split-K on bf16 MFMA with an LDS-DMA pipeline (dxgemm.hip): partials[s][M][N] =
 * A[M][k in split s] . B[N][k in split s]^T, A [M][lda] (dZ), B [N][ldb] (Wo as [d][V]), splits of
 * ceil64(ceil(K / splits)) — the same partials (and split boundaries) as cc_gemm's EPI_SPLITK NT
 * path; reduce with cc_splitk_reduce.  M, N multiples of 128, K % 8 == 0, operands < 2 GB. */
int cc_gemm_dx_splitk(const void *A, int32_t lda, const void *B, int32_t ldb, int32_t M, int32_t N,
                      int32_t K, int32_t splits, float *partials, void *stream);
/* B [N][K] bf16 (pitch ldb) -> its MFMA B-fragment image dst [N/32][ceil(K/16)][64][8] bf16 (lane L of
 * fragment (band, k step): B[32 band + (L & 31)][16 k step + 8 (L >> 5) + 0..7], zeros past K);
 * cc_pack_frag_b_size bytes.  N % 32 == 0, K % 8 == 0, 16-B aligned. */
size_t cc_pack_frag_b_size(int32_t N, int32_t K);
int cc_pack_frag_b(const void *B, int32_t N, int32_t K, int32_t ldb, void *dst, void *stream);
/* cc_gemm_dx_splitk with B given as its cc_pack_frag_b image Bp (the tall full-mode dX: Wo's
 * fragments loaded straight into registers, only dZ through LDS): the same partials bit for bit.
 * M % 128 == 0, N % 256 == 0. */
int cc_gemm_dx_splitk_pk(const void *A, int32_t lda, const void *Bp, int32_t M, int32_t N, int32_t K,
                         int32_t splits, float *partials, void *stream);
/* loss_out[0] = sum(partials[0:n]) * scale (fixed order, fp64) */
int cc_reduce_loss(const double *partials, int32_t n, double scale, double *loss_out, void *stream);

/* ----------------------------------------------------------------------------------
 * Adam (train.py:84 'adam' -> TF ResourceApplyAdam): dense over [0, n) of the flat buffers,
 * step t = state[0] + 1.  shadow (bf16) refreshed when non-NULL.
 * ---------------------------------------------------------------------------------- */
int cc_adam_dense(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t n,
                  const int64_t *state, float lr, float beta1, float beta2, float eps,
                  void *stream);
/* shadow[i] = bf16(x[i]) (round-to-nearest-even): refresh the bf16 weight shadow */
int cc_to_bf16(const float *x, uint16_t *y, int64_t n, void *stream);
/* Device step state {step, batch_in_epoch, epoch, 0}: step += 1, batch += 1, and on reaching
 * batches_per_epoch: batch = 0, epoch += 1 (on_epoch_end, generator.py:68-72).  Keeping the
 * counters on the device makes a whole training step replayable as one hipGraph. */
/* cc_adam_dense_t: cc_adam_dense over [0, n) (n % 4 == 0, shadow required) that also writes,
 * for each region k (sorted, disjoint, 4-aligned), the updated bf16 values of the row-major
 * [rows][cols] matrix at p + off transposed to dst [cols][rows] — the k-contiguous operand
 * copies (decoder Wo^T, tower W^T) the forward reads.  One launch replaces cc_adam_dense +
 * cc_transpose + cc_tower_transpose; identical values.  advance_bpe > 0 also performs
 * cc_state_advance(state, advance_bpe) once every block has read the step (state[3] is the
 * kernel's completion ticket and must be 0 between launches). */
typedef struct cc_adam_tregion {
  int64_t off;
  int32_t rows, cols;
  uint16_t *dst;
} cc_adam_tregion;
int cc_adam_dense_t(float *p, float *m, float *v, const float *g, uint16_t *shadow, int64_t n,
                    int64_t *state, float lr, float beta1, float beta2, float eps,
                    const cc_adam_tregion *regions, int32_t nregions, int64_t advance_bpe,
                    void *stream);
int cc_state_advance(int64_t *state, int64_t batches_per_epoch, void *stream);

/* ----------------------------------------------------------------------------------
 * Recommend forward (ml_recommend.py:78-87, ml_recommend_web.py:39-46), fp32, with the
 * pinned summation order of oracle/infer_ref.py (bit-exact).  R cubes per call.
 *   cc_infer_encode_fp32: zlat [R, 64]   (model.encoder(x)); row_ptr/idx = CSR of sorted unique
 *                         card ids, max_n >= the longest row; ws: cc_infer_encode_ws_size bytes.
 *   cc_infer_decode_fp32: probs [R, V]   (model.decoder(z)) — sigmoid in fp64 -> fp32;
 *                         h3_ws: [R, d] floats.
 * ---------------------------------------------------------------------------------- */
size_t cc_infer_encode_ws_size(int32_t R, int32_t d, int32_t max_n);
int cc_infer_encode_fp32(const float *params, int32_t V, int32_t d, int32_t R,
                         const int32_t *row_ptr, const int32_t *idx, int32_t max_n, void *ws,
                         float *zlat, void *stream);
int cc_infer_decode_fp32(const float *params, int32_t V, int32_t d, int32_t R,
                         const float *zlat, float *h3_ws, float *probs, void *stream);

/* ----------------------------------------------------------------------------------
 * Card similarity (src/scripts/similarity.py:19-31).  emb [V][K] fp32 = the
 * encoder on the identity (cc_infer_encode_fp32 on one-card rows).  dist_j = Keras
 * CosineSimilarity(emb[q], emb[j]) = -sum(l2_normalize(a) * l2_normalize(b)), fp32 in index
 * order without contraction; out_idx/out_dist = the N smallest by numpy argsort(kind='stable')
 * (ties -> lower index first).  dist_all (optional) receives all V distances.  N <= 4096.
 * ws: cc_similar_ws_size(V) bytes, 8-B aligned.
 * ---------------------------------------------------------------------------------- */
size_t cc_similar_ws_size(int32_t V);
int cc_similar_cards(const float *emb, int32_t V, int32_t K, int32_t q, int32_t N, int32_t *out_idx,
                     float *out_dist, float *dist_all, void *ws, void *stream);

/* ----------------------------------------------------------------------------------
 * Top-N (ml_recommend.py:87-108): rank all V probabilities descending, ties -> higher
 * index first (= numpy argsort(kind='stable')[::-1]); additions = first max(amount,1)
 * indices not in the cube; cut_vals[i] = probs[cube_idx[i]].  cube_idx: n DISTINCT card ids.
 * ws: cc_topn_workspace_size(V) bytes.
 * order == NULL: the request path (tiled multi-workgroup radix sort, 5 launches).
 * order != NULL: additionally the full ranking [V] (single-workgroup sort; tests and tools).
 * ---------------------------------------------------------------------------------- */
size_t cc_topn_workspace_size(int32_t V);
int cc_topn(const float *probs, int32_t V, const int32_t *cube_idx, int32_t n, int32_t amount,
            int32_t *additions, int32_t *n_additions, float *add_vals, float *cut_vals,
            int32_t *order, void *ws, void *stream);

/* ----------------------------------------------------------------------------------
 * One single-cube request end to end (ml_recommend.py:78-108 / ml_recommend_web.py:39-64):
 * encode + decode + top-N, no host round trip, fixed launch grids (graph-replayable).
 *   req (device):  {n, amount, ids[n]}  — the cube's sorted distinct card ids, n <= max_n
 *   res (device):  {n_add, additions[w], add_vals[w] (fp32 bits), cut_vals[n] (fp32 bits)}
 *                  with w = n_add = min(max(amount, 1), V - n)
 *   probs [V] receives the probabilities; ws: cc_recommend_ws_size(V, d) bytes, 256-B aligned.
 * ---------------------------------------------------------------------------------- */
size_t cc_recommend_ws_size(int32_t V, int32_t d);
int cc_recommend_fp32(const float *params, int32_t V, int32_t d, const int32_t *req,
                      int32_t max_n, void *ws, float *probs, int32_t *res, void *stream);

/* The same request captured once as a hipGraph: [H2D of (2 + max_n) words req_host -> req_dev]
 * + the kernels.  cc_recommend_graph_run replays it, copies res_words words of res back to
 * res_host (pinned) and waits.  Buffers stay owned by the caller and must outlive the handle. */
int cc_recommend_graph_create(const float *params, int32_t V, int32_t d, const int32_t *req_host,
                              int32_t *req_dev, int32_t max_n, void *ws, float *probs,
                              int32_t *res_dev, void **handle);
int cc_recommend_graph_run(void *handle, int32_t *res_host, int32_t res_words);
int cc_recommend_graph_destroy(void *handle);

/* ---------------------------------------------------------------- card co-occurrence graph (N1)
 * Replaces src/non_ml/utils.py:75-91 (create_adjacency_matrix, called by
 * src/non_ml/create_mtx.py:19) and the M~ normalisation of src/ml/train.py:69-71.
 * Cubes arrive as CSR lists on the device: cube c holds card ids idx[row_ptr[c] .. row_ptr[c+1])
 * (ids in [0, V), validated by the caller; duplicates collapse like the reference's dense 0/1
 * matrix).  Outputs (any subset, each row-major [V][V], device):
 *   counts   int32: |{cubes containing i and j}|                         (exact)
 *   adj      f64:   M  = counts[i,j] / counts[i,i], unseen rows 0, diag := *force_diag if given
 *                   (bit-exact with the reference's f64 M, the output/full_adj_mtx.npy format)
 *   adj_norm f32:   M~ = (M, diag := 1) / rowsum, an unseen row e_i (train.py:69-71)
 * chunk_cubes > 0 bounds the transposed 0/1 matrix held in the workspace to V x chunk bytes;
 * <= 0 processes all cubes at once.  with_counts says whether `counts` will be passed (it then
 * doubles as the accumulator across chunks). */
size_t cc_adjacency_ws_size(int32_t V, int32_t C, int32_t chunk_cubes, int32_t with_counts);
int cc_adjacency(const int32_t *row_ptr, const int32_t *idx, int32_t C, int32_t V,
                 int32_t chunk_cubes, const double *force_diag, void *ws, int32_t *counts,
                 double *adj, float *adj_norm, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CCREC_H */
