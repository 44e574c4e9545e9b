"""Device-resident DAE training step — host orchestration of the libccrec_hip kernels.

Replaces one Keras ``train_step`` of ``autoencoder.fit(generator)`` (src/ml/train.py:99-102):
    F (generator.py:74-103) -> E (model.py:35-42) -> D1 + BCE and D2 + KL (model.py:117-125,
    train.py:83-88) -> backward -> Adam (train.py:84).
Everything stays in HBM: the dataset as a CSR of card ids, the noised batch as a CSR + bitmasks,
activations in the GEMM operand dtype (bf16 or fp32), fp32 master weights + Adam moments in one
flat buffer (cubecobrarecommender_amd.layout), a bf16 shadow of the weights for the MFMA path.
torch is used only to own device memory and the stream; every computation is a HIP kernel.
"""
from dataclasses import dataclass


import numpy as np
import torch

from . import _lib as L
from .layout import Layout


@dataclass
class TrainConfig:
    V: int
    d: int = 256
    batch_size: int = 512          # per rank
    reg: float = 0.0               # train.py:86 loss_weights=[1.0, reg]
    noise: float = 0.2             # generator.py:13
    noise_std: float = 0.1         # generator.py:14
    lr: float = 1e-3               # Keras 'adam' defaults (train.py:84)
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-7
    dtype: str = 'bf16'            # GEMM operand dtype: 'bf16' (MFMA bf16), 'fp32' (exact f32 MFMA) or
    #                                'fp8' (bf16 + MX-FP8 decoder output / regulariser GEMMs, config 5)
    seed: int = 0
    rank: int = 0
    world: int = 1
    fused_tower: bool = True       # tower.hip row-block kernels (else per-layer cc_gemm launches)
    prefetch_noise: bool = True    # one process: F of step k+1 rides in step k's Adam launch
    reg_shard: bool = False        # data parallel + reg: M~ row-sharded, owner computes
    fuse_w1_adam: bool = False     # one process: TF Adam on W1 inside the W1-gradient kernel (its
    #                                gradient is then never stored; bench.py turns it on)
    wo_adam_in_tower: bool = False  # with fuse_w1_adam, bf16 d <= 256 (fused output layers): TF Adam on
    #                                the decoder output layers' tails in the tower backward launch (bench.py)
    f_in_tower: bool = False       # one process, bf16 fast chains: the NEXT step's F as extra workgroups
    #                                of the tower backward launch (cc_tower_bwd_chain_noise; every batch
    #                                buffer F writes is free by then) instead of the Adam launch (bench.py)
    wo_tower_frac: float = -1.0    # ... on this trailing fraction of each; the rest stays in the Adam + F
    #                                launch (< 0: measured per mode — 0.6 BCE only, 0.55 with the
    #                                sampled regulariser; bench.py --wo-tower-frac sweeps)
    dx_splits: int = 0             # decoder dX K-splits (0: measured default, 32 bf16 / 16 fp8)
    dx_splits_reg: int = 0         # ... of the full-mode regulariser branch (0: 4)
    dx_packed_wo: bool = True      # full-mode regulariser dX from Wo's fragment image (cc_gemm_dx_splitk_pk)
    dp_defer_out: bool = True      # data parallel: the output layers' all-gather at the next step's head
    mx8_bce_q: bool = True         # fp8: the BCE product writes dZ's MX-FP8 images (else quantiser launches)
    mx8_pair_reg_logits: bool = True   # fp8: the regulariser logits as extra blocks of the BCE product's launch
    graph_steps: int = 8           # one process: consecutive steady-state steps per hipGraph replay (step_many)
    force_dp: bool = False         # one process driving the data-parallel step (a 1-rank process group:
    #                                zero.py's collectives on device tensors; tests and the per-rank DP profile)
    dp_graph: bool = True          # data parallel over RCCL: the whole step (collectives included) as one hipGraph
    dp_f_in_adam: bool = True      # data parallel: the next step's F as extra blocks of the towers + E1
    #                                bucket's sharded Adam launch (else its own launch, cc_noise_next)
    dz_pad: bool = True            # the fused D1 kernel's dZ rows at a 64-element pitch (whole cache lines)
    w1_chunks: int = 0             # data parallel (bf16 / fp8 layout, column-slice W1 gradient): W1's
    #                                gradient launched and exchanged in this many row chunks (zero.py
    #                                reduce-scatters chunk i while chunk i+1's gradient runs); 0: by the
    #                                exchange model (tools/dp_model.py) — 1 at d <= 512, 2 above
    metrics: bool = False          # Keras metrics=['accuracy'] (train.py:87): each step counts both
    #                                outputs' categorical accuracy (TF 2.5's shape rule) on the device from
    #                                logits recomputed for the purpose (metrics.hip; take_metrics() per epoch)
    reg_by_index: bool = True      # sampled regulariser, column-slice W1 gradient: the reg rows (one card each)
    #                                enter the W1 product by index (cc_embed_grad_cs_reg: only the k-steps
    #                                that touch a tile), not as bits of a 2B-row bit matrix; bit-identical
    reg_mode: str = 'sampled'      # 'sampled': B reg rows per step drawn ∝ neg_sampler (generator.py:47-51);
    #                                'full': all |V| identity rows every step, KL(M~, D2(E(I))) as the
    #                                reference README states the objective (README.md:27)


def reg_row_shards(cdf, world):
    """Row shards of M~ for the sampled regulariser (owner computes): boundaries
    b[0..world] at equal cumulative neg_sampler mass — shard r = cards whose CDF value lies in
    (r/world, (r+1)/world] — and each shard's mass m_r = cdf[b_{r+1}-1] - cdf[b_r-1].  Rank r holds
    rows [b_r, b_{r+1}) of M~ only; every rank draws the step's world*B global reg rows (the same
    draws one process of batch world*B makes) and computes the KL terms of the rows it owns
    (cc_reg_rows), so the summed gradient is exactly the one-process gradient; equal mass balances
    the expected rows per rank."""
    cdf = np.asarray(cdf, np.float64)
    V = len(cdf)
    b = np.searchsorted(cdf, np.arange(world + 1) / float(world), side='right')
    b[0], b[world] = 0, V
    b = np.maximum.accumulate(np.minimum(b, V))
    lo_mass = np.where(b[:-1] > 0, cdf[np.maximum(b[:-1] - 1, 0)], 0.0)
    hi_mass = np.where(b[1:] > 0, cdf[np.maximum(b[1:] - 1, 0)], 0.0)
    mass = hi_mass - lo_mass
    if np.any(b[1:] <= b[:-1]) or np.any(mass <= 0):
        raise ValueError(f'reg_row_shards: a shard of {world} is empty (one card holds > 1/{world} '
                         'of the neg_sampler mass); use the replicated M~ (reg_shard=False)')
    return b.astype(np.int64), mass


def owner_capacity(mass, B, world, align=32, sigmas=6.0):
    """Reg rows each rank reserves under owner computes: the world*B global draws land in shard r
    Binomial(world*B, m_r) times; capacity = max over ranks of mean + 6 sigma (+1), rounded up to
    `align` (an overflow sets the device status bit 2 and Trainer.check_status raises)."""
    n = world * B
    m = np.asarray(mass, np.float64)
    need = np.max(n * m + sigmas * np.sqrt(n * m * (1.0 - m)) + 1.0)
    return int(min(n, int(np.ceil(need / align)) * align))


def full_rows(V, world, rank):
    """Full mode: rank r owns identity rows [r*ceil(V/W), (r+1)*ceil(V/W)) ∩ [0, V)."""
    per = -(-V // world)
    return min(V, rank * per), min(V, (rank + 1) * per)


def fused_reg_fits(hi, V, Breg):
    """cc_dec_softmax_kl_dw's 32-bit buffer extents (decreg.hip: mt_bytes < 2^31 for M~ rows up to
    `hi`, the Breg x V bf16 dZ < 2^32 bytes)."""
    return hi * V * 4 <= 0x7FFFFFFF and Breg * V * 2 <= 0xFFFFFFFF


def dx_splitk_fits(M, V, d):
    """cc_gemm_dx_splitk's operand extents (dxgemm.hip: M*V and d*V bf16 elements < 2 GB)."""
    return M * V * 2 < (1 << 31) and d * V * 2 < (1 << 31)


def _cdf(neg_sampler):
    cdf = np.cumsum(np.asarray(neg_sampler, np.float64))
    return cdf / cdf[-1]


def reg_rows_for(neg_sampler, world, rank, reg_mode='sampled'):
    """Rank's M~ row shard [lo, hi): equal neg_sampler mass (sampled) or equal rows (full)."""
    if reg_mode == 'full':
        return full_rows(len(neg_sampler), world, rank)
    b, _ = reg_row_shards(_cdf(neg_sampler), world)
    return int(b[rank]), int(b[rank + 1])


class DeviceDataset:
    """Cubes as a device CSR (sorted card ids), neg_sampler / CDF and optional M~ (fp32).
    ``reg_rows=(lo, hi)``: y_mtx holds (or is cut down to) rows [lo, hi) of M~ only — the
    row-sharded regulariser of a data-parallel rank (reg_row_shards)."""

    def __init__(self, cube_lists=None, num_cards=None, y_mtx=None, neg_sampler=None,
                 device='cuda', csr=None, reg_rows=None):
        if csr is not None:
            indptr, indices = csr
            indptr = np.asarray(indptr, np.int64)
            indices = np.asarray(indices, np.int32)
        else:
            lens = np.array([len(c) for c in cube_lists], np.int64)
            indptr = np.zeros(len(cube_lists) + 1, np.int64)
            indptr[1:] = np.cumsum(lens)
            indices = (np.concatenate([np.sort(np.asarray(c, np.int64)) for c in cube_lists])
                       .astype(np.int32) if len(cube_lists) else np.zeros(0, np.int32))
        self.V = int(num_cards)
        self.C = len(indptr) - 1
        self.max_n = int(np.max(np.diff(indptr))) if self.C else 0
        self.cube_ptr = torch.from_numpy(indptr).to(device)
        self.cube_idx = torch.from_numpy(indices).to(device)
        if neg_sampler is None:
            if y_mtx is None:
                raise ValueError('need y_mtx (M~) or neg_sampler')
            neg_sampler = _neg_sampler(y_mtx)
        ns = np.asarray(neg_sampler, np.float64)
        cdf = _cdf(ns)
        self.neg_sampler_host = ns
        self.cdf_host = cdf
        self.neg_sampler = torch.from_numpy(ns).to(device)
        self.cdf = torch.from_numpy(cdf).to(device)
        # CDF search guide table (2^16 + 1 entries, 256 KB): with Zipf-like popularity the tail
        # cards share buckets, and each extra entry per bucket is one more dependent fp64 load in
        # F's add draws (measured at 2^12: the add phase 3.5 us mean, 7.9 us worst per cube)
        self.guide_log2 = 16
        guide = np.searchsorted(cdf, np.arange((1 << self.guide_log2) + 1) / float(1 << self.guide_log2), side='right')
        self.guide = torch.from_numpy(guide.astype(np.int32)).to(device)
        self.y_reg = None
        self.reg_rows = None
        if y_mtx is not None:
            y = y_mtx if torch.is_tensor(y_mtx) else torch.from_numpy(np.asarray(y_mtx, np.float32))
            lo, hi = reg_rows if reg_rows is not None else (0, self.V)
            if y.shape[0] == self.V and (lo, hi) != (0, self.V):
                y = y[lo:hi]
            if y.shape != (hi - lo, self.V):
                raise ValueError(f'y_mtx rows {tuple(y.shape)}: expected ({hi - lo}, {self.V})')
            self.y_reg = y.to(device=device, dtype=torch.float32).contiguous()
            self.reg_rows = (int(lo), int(hi))


def branches_of(use_reg):
    return ('decoder', 'decoder_for_reg') if use_reg else ('decoder',)


def _neg_sampler(y_mtx):
    """generator.py:30: neg_sampler = M~.sum(0) / M~.sum() (float64)."""
    if torch.is_tensor(y_mtx):
        y = y_mtx.to(torch.float64)
        return (y.sum(0) / y.sum()).cpu().numpy()
    y = np.asarray(y_mtx, np.float64)
    return y.sum(0) / y.sum()


class Trainer:
    def __init__(self, cfg: TrainConfig, data: DeviceDataset, params_flat=None, device='cuda'):
        L.lib()  # fail loudly before allocating anything
        self.cfg, self.data = cfg, data
        V, d, B = cfg.V, cfg.d, cfg.batch_size
        assert data.V == V, 'dataset V mismatch'
        assert d % 64 == 0 and (d // 64) & (d // 64 - 1) == 0, 'd must be 64 * 2^k'
        self.dev = torch.device(device)
        # data-parallel: gradient buckets aligned to world*64 so every rank owns an equal shard
        self.std_layout = Layout(V, d)
        self.dp = cfg.world > 1 or cfg.force_dp    # zero.py's sharded step (buckets, collectives)
        # (with a bf16 shadow the biases are grouped so zero.py all-gathers the kernels' bf16 shadow)
        self.layout = (Layout(V, d, align=cfg.world * 64, group_biases=cfg.dtype in ('bf16', 'fp8'),
                              w1_chunks=(1 if cfg.reg_mode == 'full' else cfg.w1_chunks if cfg.w1_chunks > 0
                                         else 1 if d <= 512 else 2))
                       if self.dp else self.std_layout)
        self.use_reg = cfg.reg > 0
        if self.use_reg and data.y_reg is None:
            raise ValueError('reg > 0 needs the M~ matrix on the device')
        if cfg.reg_mode not in ('sampled', 'full'):
            raise ValueError(f"reg_mode {cfg.reg_mode!r}: 'sampled' or 'full'")
        W = cfg.world
        self.full_reg = self.use_reg and cfg.reg_mode == 'full'
        self.owner = self.use_reg and not self.full_reg and cfg.reg_shard and self.dp
        ralign = 128 if cfg.dtype == 'fp8' else 32
        # regulariser rows of this rank: rows [B, B + Breg) of every row-indexed buffer.
        #   sampled: B draws per step (slot b of cube b), dz weight reg/B;
        #   owner (data parallel, M~ row-sharded): the world*B global draws that fall in this
        #     rank's shard, padded to a static capacity, masked rows reg_idx = -1; weight reg/B
        #     (the zero.py average over ranks makes it reg/(world*B) per global row);
        #   full: identity rows [lo, hi) (all of V on one GPU), weight reg*world/V.
        self.reg_rows = (0, V)
        self.Breg = B if self.use_reg else 0
        self.kl_row_scale, self.kl_loss_scale = cfg.reg / B, 1.0 / B
        if self.full_reg:
            self.reg_rows = full_rows(V, W, cfg.rank)
            n = self.reg_rows[1] - self.reg_rows[0]
            self.Breg = -(-n // ralign) * ralign
            self.kl_row_scale, self.kl_loss_scale = cfg.reg * W / V, W / V
        elif self.owner:
            bnd, mass = reg_row_shards(data.cdf_host, W)
            self.reg_rows = (int(bnd[cfg.rank]), int(bnd[cfg.rank + 1]))
            self.Breg = owner_capacity(mass, B, W, align=ralign)
        self.R = B + self.Breg
        # the sampled reg rows by index in the W1 gradient (cc_embed_grad_cs_reg; its column-slice
        # path runs exactly when the fused towers and the MFMA W1 gradient do: bf16 / fp8, d % 128)
        # (not with f_in_tower: the next step's F, drawn in the tower backward launch, rewrites the reg
        # cards before the W1 gradient reads them; the bit matrix is not rewritten by F)
        self.reg_by_index = bool(cfg.reg_by_index and self.use_reg and not self.full_reg
                                 and cfg.dtype in ('bf16', 'fp8') and cfg.fused_tower and B % 32 == 0
                                 and d <= 1024 and d % 128 == 0 and 0 < self.Breg <= 512 and not cfg.f_in_tower)
        # rows of the MFMA W1-gradient product (its bit matrix): the cubes only when the regulariser
        # rows enter by index (full mode: cc_embed_identity_add; sampled: cc_embed_grad_cs_reg)
        self.xt_rows = B if (self.full_reg or self.reg_by_index) else self.R
        self.reg_weight = 1.0
        if self.use_reg and data.reg_rows != self.reg_rows:
            if data.reg_rows != (0, V):
                raise ValueError(f'dataset holds M~ rows {data.reg_rows}, rank needs {self.reg_rows}')
            lo, hi = self.reg_rows
            data.y_reg, data.reg_rows = data.y_reg[lo:hi].contiguous(), self.reg_rows
        if cfg.dtype not in ('bf16', 'fp32', 'fp8'):
            raise ValueError(f'dtype {cfg.dtype!r}: bf16, fp32 or fp8')
        self.mx8 = cfg.dtype == 'fp8'
        self.dtype = L.CC_F32 if cfg.dtype == 'fp32' else L.CC_BF16
        self.tdt = torch.float32 if cfg.dtype == 'fp32' else torch.bfloat16
        if self.mx8 and (d % 128 or self.R % 128 or B % 32):
            raise ValueError('fp8 (MX) decoder GEMMs need d and the row count (B, 2B with reg) multiples of 128')
        P = self.layout.total
        f32 = dict(device=self.dev, dtype=torch.float32)
        self.params = torch.zeros(P, **f32)
        if params_flat is not None:   # given in the standard (cc_param_layout) layout
            self.load_standard(self.params, params_flat)
        self.m = torch.zeros(P, **f32)
        self.v = torch.zeros(P, **f32)
        self.grads = torch.zeros(P, **f32)
        self.shadow = torch.zeros(P, device=self.dev, dtype=torch.bfloat16) if self.dtype == L.CC_BF16 else None
        self.refresh_shadow()
        self.state = torch.zeros(4, device=self.dev, dtype=torch.int64)   # {step, batch, epoch, ticket}
        self.tickets = torch.zeros(4, device=self.dev, dtype=torch.int32)  # last-block hand-offs
        self.x_cap = max(1, data.max_n + int(data.max_n * 0.8) + 1)
        R, VW, XW = self.R, (V + 31) // 32, (self.xt_rows + 31) // 32
        i32 = dict(device=self.dev, dtype=torch.int32)
        self.x_cnt = torch.zeros(R, **i32)
        self.x_idx = torch.zeros(R, self.x_cap, **i32)
        self.y_bits = torch.zeros(B, VW, **i32)
        self.xt_bits = torch.zeros(V, XW, **i32)
        self.reg_idx = torch.zeros(max(self.Breg, 1), **i32)
        self.status = torch.zeros(1, **i32)
        T = dict(device=self.dev, dtype=self.tdt)
        self.H1 = torch.zeros(R, d, **T)
        self.H2 = torch.zeros(R, 256, **T)
        self.H3 = torch.zeros(R, 128, **T)
        self.Zl = torch.zeros(R, 64, **T)
        self.D1 = torch.zeros(R, 128, **T)
        self.D2 = torch.zeros(R, 256, **T)
        self.D3 = torch.zeros(R, d, **T)
        self.dZout = torch.zeros(R, V, **T)       # rows [0,B): D1 dZ, rows [B,2B): D2 dZ
        self.gD3 = torch.zeros(R, d, **T)
        self.gD2 = torch.zeros(R, 256, **T)
        self.gD1 = torch.zeros(R, 128, **T)
        self.gZl = torch.zeros(R, 64, **T)
        self.gH3 = torch.zeros(R, 128, **T)
        self.gH2 = torch.zeros(R, 256, **T)
        self.gPre1 = torch.zeros(R, d, **f32)
        self.Z2 = None             # materialised fp32 D2 logits (the unfused regulariser path only)
        self.splits = max(1, min(cfg.dx_splits or (16 if cfg.dtype == 'fp8' else 32), V // 512))   # decoder dX: K = V (fp8: 256 x 256 tiles, 16 splits measured best)
        # the regulariser branch's dX: M = Breg rows; with thousands of rows (full mode) the output
        # tiles alone fill the chip — no split-K
        # full-mode regulariser (~|V| rows): 2 K-splits (tools/micro/dx_full_micro.py at |V| = 22,000:
        # 1 split 643 us, 2 or 4 splits 515 us, the library GEMM 391-399 us)
        # (the 128 x 256-tile kernel of dxgemm.hip for tall M: 4 splits)
        self.splits_reg = self.splits if self.Breg <= 1024 else (cfg.dx_splits_reg or 4)
        self.tsplits = max(1, min(8, B // 128))             # tower dW: K = rows (B or 2B)
        self.split_buf = torch.zeros(max(self.splits * B * d, self.splits_reg * self.Breg * d,
                                         2 * self.tsplits * max(d, 256) * 256), **f32)
        self.cs_buf = torch.zeros(2 * self.tsplits * max(d, 256), **f32)
        tiles = ((B + 63) // 64) * ((V + 63) // 64)
        self.bce_part = torch.zeros(tiles, device=self.dev, dtype=torch.float64)
        self.kl_part = torch.zeros(max(self.Breg, 1), device=self.dev, dtype=torch.float64)
        self.id_ws = (torch.zeros(int(L.lib().cc_embed_identity_ws(self.Breg, d)) // 4 + 1, **f32)
                      if self.full_reg else None)
        self.loss_dev = torch.zeros(2, device=self.dev, dtype=torch.float64)
        # fused 32-row-block towers (tower.hip) when the widths fit; generic GEMMs otherwise
        self.fused_tower = cfg.fused_tower and (B % 32 == 0) and d <= (1024 if self.dtype == L.CC_BF16 else 256)
        # bf16 path: the W1 gradient on MFMA (cc_embed_grad_mfma) from dPre1^T bf16 [d][RP]
        # written by the tower backward chain (columns R..RP-1 stay zero)
        self.embed_mfma = self.dtype == L.CC_BF16 and self.fused_tower and d % 128 == 0 and self.xt_rows <= 2048
        self.RP = (R + 63) // 64 * 64
        # decoder dX on the LDS-DMA pipelined split-K kernel (dxgemm.hip; other dtypes: gemm.hip's)
        self.dx_glds = self.dtype == L.CC_BF16
        self.WoP = None   # the full-mode regulariser's Wo as its MFMA fragment image (below)
        # D1 output layer fused (logits + BCE + dZ + dWo, csrc/decout.hip) where its shape fits
        self.fused_out = (self.dtype == L.CC_BF16 and self.fused_tower and not self.mx8 and d in (128, 256, 512)
                          and B in (128, 256, 512))
        # the fused D1 kernel's dZ rows at a pitch of whole 64-element (128-B) groups: at |V| = 22,000
        # the natural pitch (44,000 B) starts every other row mid-line, so a wave's 64-B row segments
        # straddle lines shared with the next row / the next 96-column slice; the dX product reads
        # dZ at the padded pitch (measured r04u: 154.0 / 154.2 -> 153.3 / 152.5 us/step, FETCH_SIZE
        # of the kernel unchanged)
        self.dz1_ld = V
        self.dZ1 = None
        if self.fused_out:
            self.dz1_ld = -(-V // 64) * 64 if cfg.dz_pad else V
            self.dZ1 = torch.zeros(B, self.dz1_ld, **T)
        self.gPre1T = torch.zeros(d, self.RP, **T) if self.embed_mfma else None
        if self.mx8 and not self.fused_tower:
            raise ValueError('fp8 needs the fused towers (fused_tower=True, B % 32 == 0)')
        self.wpack = self.D3p = self.D3tp = self.hpt = self.gpt = self.gpre1p = self.eg_tickets = None
        if self.fused_tower:
            self.tower_layers = ('encoder/encoded_2', 'encoder/encoded_3', 'encoder/bottleneck',
                                 'decoder/decoded_1', 'decoder/decoded_2', 'decoder/decoded_3',
                                 'decoder_for_reg/decoded_1', 'decoder_for_reg/decoded_2',
                                 'decoder_for_reg/decoded_3')
            sizes = [int(np.prod(self.layout.shape(n + '/kernel'))) for n in self.tower_layers]
            self.wt_off = np.concatenate([[0], np.cumsum([(n + 63) // 64 * 64 for n in sizes])])
            self.wt = torch.zeros(int(self.wt_off[-1]), **T)
            # fragment-packed forward/backward weight images for the bf16 tower kernels (d <= 256:
            # fast, 256 < d <= 1024: wide; written with wt by cc_tower_transpose and by the Adam
            # launch; the opt-in fused Adam writes only wt)
            pack = self.dtype == L.CC_BF16 and d <= 1024
            self.wpack = torch.zeros(2, int(self.wt_off[-1]), **T) if pack else None
            # ... and D3 as packed operand images of the fused D1 output kernel (cc_dec_bce_dw)
            self.D3p = torch.zeros(R * d, **T) if pack else None
            self.D3tp = torch.zeros(d * R, **T) if pack else None
            # ... and every tower layer's input / output-gradient as packed transposed images
            # (the dW kernel's MFMA operands): H widths d,256,128,64,128,256; G 256,128,64,128,256,d
            self.hpt = [torch.zeros(R * w, **T) for w in (d, 256, 128, 64, 128, 256)] if pack else None
            self.gpt = [torch.zeros(R * w, **T) for w in (256, 128, 64, 128, 256, d)] if pack else None
            # dPre1 as packed transposed fragments (the W1 gradient's B operand; rows past R zero)
            self.gpre1p = (torch.zeros(d * self.RP, **T) if pack and self.embed_mfma and d == 256
                           else None)
            # the W1 gradient by column slices (cc_embed_grad_cs; without the MFMA operands: the row kernels):
            # one zeroed ticket per row chunk, left zero by every call
            self.eg_tickets = (torch.zeros(max(1, int(L.lib().cc_embed_grad_cs_tickets(V, d, self.xt_rows))),
                                           device=self.dev, dtype=torch.int32)
                               if (self.gpre1p is not None or self.embed_mfma)
                               else None)
            assert not self.reg_by_index or self.eg_tickets is not None, 'reg_by_index needs the column-slice W1 gradient'
            slab = int(L.lib().cc_tower_slab_elems(d))
            self.slab = torch.zeros((R // 32) * slab, **f32)
            # D2 output layer fused (logits twice -> softmax -> KL -> dZ -> dWo, csrc/decreg.hip): bf16,
            # d in {128, 256, 512} with the packed D3 images (the same shape class as the fused D1 kernel)
            # (its buffer descriptors address M~ up to row hi and the Breg x V bf16 dZ with 32-bit
            # extents: larger card pools fall back to the Z2 path instead of failing)
            self.fused_reg = (self.use_reg and self.D3p is not None and not self.mx8 and d in (128, 256, 512)
                              and self.Breg % 32 == 0 and fused_reg_fits(self.reg_rows[1], V, self.Breg))
            # decoder operands kept k-contiguous: D3^T (tower fwd), dZ^T (BCE epilogue), Wo^T shadow
            self.D3t = torch.zeros(d, R, **T)
            self.dZt = [torch.zeros(V, n, **T) if not (k == 1 and self.fused_reg) else None
                        for k, n in enumerate(self.branch_rows())]   # [branch][V][rows]
            self.WoT = torch.zeros(len(branches_of(self.use_reg)), V, d, **T)
            # the full-mode regulariser's dX takes Wo as its MFMA B-fragment image (cc_pack_frag_b,
            # refreshed with the other decoder operands after each update; cc_gemm_dx_splitk_pk)
            if (self.full_reg and self.fused_reg and self.dx_glds and d % 256 == 0 and V % 8 == 0
                    and self.Breg % 128 == 0 and cfg.dx_packed_wo):
                self.WoP = torch.zeros(int(L.lib().cc_pack_frag_b_size(d, V)) // 2, **T)
            if self.mx8:   # MX-FP8 operand images of the decoder output layers (csrc/mx8.hip)
                nbr, u8 = len(branches_of(self.use_reg)), dict(device=self.dev, dtype=torch.uint8)
                self.Vp = (V + 127) // 128 * 128
                self.WoT8 = torch.zeros(nbr, V, d, **u8)                  # fwd B operand [V][d]
                self.WoT8s = torch.zeros(nbr, V, d // 32, **u8)
                self.Wo8 = torch.zeros(nbr, d, self.Vp, **u8)             # dX B operand [d][Vp]
                self.Wo8s = torch.zeros(nbr, d, self.Vp // 32, **u8)
                self.D3q = torch.zeros(R, d, **u8)                        # fwd A operand
                self.D3qs = torch.zeros(R, d // 32, **u8)
                self.D3tq = torch.zeros(d, R, **u8)                       # dW A operand (K = rows)
                self.D3tqs = torch.zeros(d, R // 32, **u8)
                self.dZq = torch.zeros(R, self.Vp, **u8)                  # dX A operand
                self.dZqs = torch.zeros(R, self.Vp // 32, **u8)
                self.dZtq = [torch.zeros(V, n, **u8) for n in self.branch_rows()]   # dW B operand (K = rows)
                self.dZtqs = [torch.zeros(V, n // 32, **u8) for n in self.branch_rows()]
            self.targs = self._tower_args()
            # config 5 on the wide chains: the tower forward writes D3's MX-FP8 images itself (two
            # quantiser launches less per step)
            self.d3q_in_tower = self.mx8 and d > 256 and self.wpack is not None and R % 32 == 0
            # the BCE product makes dZ's MX-FP8 images and the bias gradient in its epilogue
            # (cc_gemm_mx8_bce_q: B % 32 == 0, B <= 512); mx8_bce_q=False keeps the quantiser launches
            self.mx8_bce_q = self.mx8 and B % 32 == 0 and B <= 512 and cfg.mx8_bce_q
            if self.d3q_in_tower:
                t = self.targs
                t.d3q, t.d3qs = self.D3q.data_ptr(), self.D3qs.data_ptr()
                t.d3tq, t.d3tqs = self.D3tq.data_ptr(), self.D3tqs.data_ptr()
            self.transpose_tower()
        else:
            self.targs = None
            self.d3q_in_tower = False
            self.mx8_bce_q = False
        if not self.fused_tower:
            self.fused_reg = False
        if self.use_reg and not self.fused_reg:
            self.Z2 = torch.zeros(self.Breg, V, **f32)
        # config 5: the regulariser logits ride in the BCE product's launch (cc_gemm_mx8_bce_q2)
        self.reg_logits_paired = (self.mx8_bce_q and self.use_reg and not self.fused_reg and self.fused_tower
                                  and cfg.mx8_pair_reg_logits)
        if self.fused_reg:
            lo, hi = self.reg_rows
            self.tsum = torch.zeros(hi - lo, 2, **f32)    # per M~ row {sum t, sum t ln t} (t clipped), once
            L.call('cc_kl_tsum', L.ptr(data.y_reg), hi - lo, V, L.ptr(self.tsum), L.stream_ptr())
            self.kl_ws = torch.zeros(int(L.lib().cc_dec_kl_ws_size(self.Breg, V)) // 4 + 4, **f32)
            self.kl_flags = 0   # cc_dec_kl_args.flags (tests: the A/B of decreg.hip's alternative full-mode paths)
            self.kl_part = torch.zeros(max(int(L.lib().cc_dec_kl_blocks(V)), 1), device=self.dev,
                                       dtype=torch.float64)
        if self.full_reg:
            self._init_full_rows()
        # metrics=['accuracy']: {output 1 correct rows, output 2 correct rows, output 2 rows} summed on
        # the device
        self.acc_counts = None
        if cfg.metrics:
            self.acc_counts = torch.zeros(3, device=self.dev, dtype=torch.int64)
            self.Z1m = torch.zeros(B, V, **f32)
            if self.use_reg:
                # (full mode's |V| identity rows go through a bounded buffer in row chunks)
                self.Z2m = self.Z2 if self.Z2 is not None else torch.zeros(min(self.Breg, 1024), V, **f32)
                lo, hi = self.reg_rows       # argmax of every resident M~ row (y_true), once
                self.t_argmax = torch.zeros(hi - lo, device=self.dev, dtype=torch.int32)
                L.call('cc_row_argmax', L.ptr(data.y_reg), V, hi - lo, V, L.ptr(self.t_argmax), L.stream_ptr())
        # F for the next step in the Adam launch (cc_adam_noise): Adam is HBM-bound, F latency-
        # bound; F then leaves the forward's critical path.  noise_ready: the batch buffers
        # already hold the batch the next forward_backward consumes.
        self.prefetch = cfg.prefetch_noise and not self.dp
        # data parallel: F of the next step is its own launch (cc_noise_next) beside the exchange of
        # the last gradient buckets (zero.py after_b), off the next forward's critical path
        self.prefetch_dp = cfg.prefetch_noise and self.dp
        # one process: F (in the Adam launch) writes its x rows as bitmasks and the next E1 gather
        # launch bit-transposes them into the W1-gradient bitmask (cc_embed_gather_fwd_xt) — F's
        # scattered xt atomics queued behind the Adam streams (measured: the Adam + F launch
        # 40.5 -> 36.9 us without them; the same atomics in the gather cost it 13 us)
        self.xt_in_gather = self.prefetch and self.dtype == L.CC_BF16
        # (F's x rows as bitmasks [R][ceil(V/32)]; rows F does not draw stay zero)
        self.x_bits = (torch.zeros(self.R, (cfg.V + 31) // 32, device=self.dev, dtype=torch.int32)
                       if self.xt_in_gather else None)
        # ... in the tower forward launch instead when its fast kernel runs (d <= 256): its 16-32
        # chain blocks leave the other CUs idle (measured: in the gather launch the transpose
        # blocks cost it 2-3 us)
        self.xt_in_tower = self.xt_in_gather and self.targs is not None and cfg.d <= 256
        if self.xt_in_tower:
            self.targs.x_bits, self.targs.xt_bits = self.x_bits.data_ptr(), self.xt_bits.data_ptr()
            self.targs.xt_V, self.targs.xt_rows = cfg.V, self.xt_rows
        # the fused D1 kernel's target masks as an image in accumulator-register row order
        # (cc_tower_args.y_img), transposed from F's y words by the tower forward launch's extra
        # blocks: the D1 epilogue then loads a tile's 16 lane masks with two scalar loads
        self.y_img = None
        if (self.fused_out and self.fused_tower and self.targs is not None and self.dtype == L.CC_BF16
                and cfg.d <= 256):
            self.y_img = torch.zeros((cfg.V + 31) // 32 * B, device=self.dev, dtype=torch.int32)
            self.targs.y_bits, self.targs.y_img, self.targs.y_V = self.y_bits.data_ptr(), self.y_img.data_ptr(), cfg.V
        # one process, packed tower images: the Adam + F launch also rewrites the tower kernels'
        # packed images and advances the step counters (cc_adam_noise_pack) — the next step
        # starts without a counters/transposes launch
        self.adam_packs = self.prefetch and self.wpack is not None
        # TF Adam on W1 in the W1-gradient kernel's epilogue (cc_embed_grad_cs_adam): the main Adam
        # launch then starts after W1 (W1 is the first tensor of the layout).  One process only
        # (DP reduces the gradient first), the column-slice kernel, not the full-mode regulariser
        # (its identity rows add to the W1 gradient after that kernel).
        self.w1_off = self.layout.offset('encoder/encoded_1/bias')   # = W1's padded size
        self.fuse_w1 = (cfg.fuse_w1_adam and self.adam_packs and self.eg_tickets is not None and not self.full_reg
                        and self.layout.offset('encoder/encoded_1/kernel') == 0)
        self.adam_pack = self._adam_pack_desc() if self.adam_packs else None
        # TF Adam on the decoder output layers (Wo, bo, and with the sampled regulariser Wo_reg, bo_reg:
        # ~96% of the parameters after W1) in extra workgroups of the tower backward launch
        # (cc_tower_bwd_chain_adam): their gradients are final after the output-layer kernels, the dX
        # products have read their bf16 shadows, and the 16-32 latency-bound chain blocks leave the
        # other CUs idle.  Only their trailing wo_tower_frac: the main Adam launch (which also runs
        # the next step's F, latency-bound too) keeps the rest to stream beside F.  wo_ranges: the
        # tower launch's [lo, hi) flat ranges; rest_ranges: the Adam launch's (W1 end onwards).
        self.wo_ranges, self.rest_ranges = None, None
        if (cfg.wo_adam_in_tower and self.fuse_w1 and self.fused_out and (not self.use_reg or self.fused_reg)
                and self.targs is not None and self.dtype == L.CC_BF16 and cfg.d <= 256):
            frac = cfg.wo_tower_frac if cfg.wo_tower_frac >= 0 else (0.55 if self.use_reg else 0.6)
            frac = min(max(float(frac), 0.0), 1.0)
            lay = self.layout
            spans = [(lay.offset('decoder/reconstruct/kernel'), lay.main_total)]
            if self.use_reg:
                spans.append((lay.offset('decoder_for_reg/reconstruct/kernel'), lay.total))
            wo = [(hi - int((hi - lo) * frac) // 256 * 256, hi) for lo, hi in spans]
            if all(a < b for a, b in wo):
                self.wo_ranges = wo
                rest, lo = [], self.w1_off
                for a, b in wo:        # the complement inside [W1 end, end of the Adam range)
                    rest.append((lo, a))
                    lo = b
                self.rest_ranges = rest
        self.wo_range = self.wo_ranges[0] if self.wo_ranges else None   # (tests: is the placement on)
        # the next step's F in the tower backward launch: one process with F prefetched (xt bits by
        # the tower forward's transpose, so F sets none the W1 gradient still reads), the packed
        # Adam launch, the fast bf16 chains
        self.f_in_tower = (cfg.f_in_tower and self.adam_packs and self.xt_in_tower and self.fused_tower
                           and self.dtype == L.CC_BF16 and cfg.d <= 256 and not self.full_reg)
        self._adv_deferred = False   # the previous step's counter advance rides in the E1 gather
        self.noise_ready = False
        self.host_batch = False      # load_batch(): the next step runs on a host-given batch
        self.perms = None
        self.batches_per_epoch = max(1, data.C // (B * cfg.world))   # generator.py:36 (__len__)
        self.graphs = None
        self.g_multi, self.multi_n, self.multi_acc = None, 0, None   # capture(): step_many's graph
        self.g_multi_sizes = {}      # capture(): step_many's graphs by step count (graph_steps and halves)
        self.g_dp = self.g_dp_nocomm = None   # capture(): the whole data-parallel step (RCCL inside)
        self.sharded = None
        self.pending_rest = False    # one process: step k's counters/transposes run at the head
        #                              of step k+1's forward graph (one graph launch less per step)
        self.side = torch.cuda.Stream(device=self.dev)   # dW / slab reduce / losses / transposes
        # the side-stream work (output-layer dW, slab reduces) as graph branches: measured slower than
        # keeping it on the one stream (r03: the tower dW beside the W1 gradient, 166.5 -> 181.7 us
        # per step — every kernel of the graph got slower), so _fork / _join only mark where it could
        # branch
        self.overlap = False
        self.timing = False          # bench.py: HIP events around the main kernels
        self.events = {}
        # zero.py (one captured data-parallel step): called on the launching stream once the decoder
        # output layer's gradient is final (hook_out) and once the branch's dX product no longer
        # reads its bf16 shadow (hook_dx), so that bucket's reduce-scatter starts before dX
        self.hook_out = self.hook_dx = None
        # ... and (a deferred output-layer all-gather, zero.py) right before the forward's D1 launch
        self.hook_d1 = None
        # ... and per gradient bucket finalised inside forward_backward_b (the towers, each W1 row
        # chunk): name -> callable, fired once on the launching stream right after the bucket's
        # last kernel
        self.bucket_hooks = {}
        # the data-parallel bf16 / fp8 layout: both output layers are one early bucket, so its
        # exchange waits for the regulariser branch's output-layer gradient and dX too
        self.early_reg_out = self.dp and self.layout.group_biases and self.use_reg

    def branch_rows(self):
        """Rows of each decoder branch: B cubes, then Breg regulariser rows."""
        return (self.cfg.batch_size, self.Breg) if self.use_reg else (self.cfg.batch_size,)

    def branches(self):
        """[(layer prefix, (r0, r1))] of the decoder branches in row order."""
        B = self.cfg.batch_size
        out = [('decoder', (0, B))]
        if self.use_reg:
            out.append(('decoder_for_reg', (B, B + self.Breg)))
        return out

    def _init_full_rows(self):
        """Full mode: the regulariser rows are the static identity rows lo..hi-1 (x row = {card},
        reg_idx = card); padding rows reg_idx -1, x_cnt 0.  Nothing redraws them per step."""
        B, (lo, hi) = self.cfg.batch_size, self.reg_rows
        n = hi - lo
        ids = torch.full((self.Breg,), -1, dtype=torch.int32)
        ids[:n] = torch.arange(lo, hi, dtype=torch.int32)
        self.reg_idx.copy_(ids)
        cnt = torch.zeros(self.Breg, dtype=torch.int32)
        cnt[:n] = 1
        self.x_cnt[B:].copy_(cnt)
        self.x_idx[B:, 0].copy_(ids.clamp(min=0))

    def check_status(self):
        """Raise on device-side error flags (bit 1: a noised cube overflowed x_cap; bit 2: more
        owned regulariser draws than the owner-computes capacity)."""
        st = int(self.status.item())
        if st:
            raise RuntimeError(f'device status {st}: ' + ('x_cap overflow ' if st & 1 else '') +
                               ('owner-computes reg capacity overflow' if st & 2 else ''))

    def _tick(self, name, stream=None):
        """Record a HIP event on the launching stream (bench timing); returns a closer."""
        if not self.timing:
            return lambda: None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)

        def close():
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(stream)
            self.events.setdefault(name, []).append((e0, e1))
        return close

    # ---- a second stream for work off the critical path (graph branches when captured)
    def _fork(self):
        """The side stream starts after everything issued so far on the current stream."""
        if not self.overlap:
            return L.stream_ptr(None)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.side.wait_event(ev)
        return L.stream_ptr(self.side)

    def _join(self):
        if not self.overlap:
            return
        ev = torch.cuda.Event()
        ev.record(self.side)
        torch.cuda.current_stream().wait_event(ev)

    def kernel_times_ms(self):
        """Average duration (ms) per instrumented kernel over the recorded launches."""
        torch.cuda.synchronize()
        return {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in self.events.items()}

    # ------------------------------------------------------------------ helpers
    def w(self, name):
        """Operand pointer of a weight: bf16 shadow or fp32 master."""
        src = self.shadow if self.shadow is not None else self.params
        return L.ptr(src[self.layout.offset(name):])

    def pf(self, name):
        return L.ptr(self.params[self.layout.offset(name):])

    def gp(self, name):
        return L.ptr(self.grads[self.layout.offset(name):])

    def _tower_args(self):
        t = L.TowerArgs(dtype=self.dtype, d=self.cfg.d, B=self.cfg.batch_size, R=self.R)
        src = self.shadow if self.shadow is not None else self.params
        for l, name in enumerate(self.tower_layers):
            t.w[l] = src[self.layout.offset(name + '/kernel'):].data_ptr()
            t.wt[l] = self.wt[int(self.wt_off[l]):].data_ptr()
            if self.wpack is not None:
                t.wpf[l] = self.wpack[0, int(self.wt_off[l]):].data_ptr()
                t.wpb[l] = self.wpack[1, int(self.wt_off[l]):].data_ptr()
            t.b[l] = self.params[self.layout.offset(name + '/bias'):].data_ptr()
            t.gw[l] = self.grads[self.layout.offset(name + '/kernel'):].data_ptr()
            t.gb[l] = self.grads[self.layout.offset(name + '/bias'):].data_ptr()
        for a, buf in enumerate((self.H1, self.H2, self.H3, self.Zl, self.D1, self.D2, self.D3)):
            t.act[a] = buf.data_ptr()
        t.act6t = self.D3t.data_ptr()
        if self.D3p is not None and (self.fused_out or self.fused_reg):   # the fused output kernels' operands
            t.act6p, t.act6tp = self.D3p.data_ptr(), self.D3tp.data_ptr()
        if self.gpre1p is not None:
            t.gpre1p = self.gpre1p.data_ptr()
        if getattr(self, 'hpt', None) is not None:
            for a in range(6):
                t.hpt[a], t.gpt[a] = self.hpt[a].data_ptr(), self.gpt[a].data_ptr()
        t.gD3 = self.gD3.data_ptr()
        for a, buf in enumerate((self.gH2, self.gH3, self.gZl, self.gD1, self.gD2)):
            t.gact[a] = buf.data_ptr()      # dPre of e2, e3, e4, d1, d2
        t.gpre1 = self.gPre1.data_ptr()
        t.gpre1t = self.gPre1T.data_ptr() if self.gPre1T is not None else None
        t.slab = self.slab.data_ptr()
        return t

    def _adam_pack_desc(self):
        layers = 9 if self.use_reg else 6
        pk = L.AdamPack(n=layers)
        for l, name in enumerate(self.tower_layers[:layers]):
            K, N = self.layout.shape(name + '/kernel')
            pk.K[l], pk.N[l] = K, N
            pk.off[l] = self.layout.offset(name + '/kernel') - (self.w1_off if self.fuse_w1 else 0)
            pk.wpf[l] = self.wpack[0, int(self.wt_off[l]):].data_ptr()
            pk.wpb[l] = self.wpack[1, int(self.wt_off[l]):].data_ptr()
        return pk

    def refresh_decoder_operands(self, s):
        """Decoder output-layer operands from the current (bf16 shadow) weights Wo [d][V]: Wo^T
        (bf16), or with fp8 the MX-FP8 images Wo^T [V][d] (forward) and Wo [d][Vp] (dX)."""
        d, V = self.cfg.d, self.cfg.V
        for k, pre in enumerate(branches_of(self.use_reg)):
            if k == 0 and self.fused_out:
                continue    # cc_dec_bce_dw reads Wo itself: no Wo^T copy for the D1 branch
            if k == 1 and self.fused_reg:   # cc_dec_softmax_kl_dw reads Wo itself
                if self.WoP is not None:     # ... the dX product its fragment image
                    L.call('cc_pack_frag_b', self.w(pre + '/reconstruct/kernel'), d, V, V, L.ptr(self.WoP), s)
                continue
            if self.mx8:   # both images from one read of Wo (cc_quant_mx8_both)
                L.call('cc_quant_mx8_both', L.CC_BF16, self.w(pre + '/reconstruct/kernel'), d, V, V,
                       L.ptr(self.WoT8[k]), d, L.ptr(self.WoT8s[k]), L.ptr(self.Wo8[k]), self.Vp,
                       L.ptr(self.Wo8s[k]), s)
            else:
                L.call('cc_transpose', self.dtype, self.w(pre + '/reconstruct/kernel'), d, V,
                       L.ptr(self.WoT[k]), s)

    def transpose_tower(self, stream=None):
        """Refresh the transposed operand copies (tower W^T, decoder Wo^T) from the current weights."""
        if self.fused_tower:
            s = L.stream_ptr(stream)
            L.call('cc_tower_transpose', L.C.byref(self.targs), s)
            self.refresh_decoder_operands(s)

    def refresh_shadow(self):
        """Re-derive the bf16 shadow (and the transposed tower operands) from the fp32 master."""
        if self.shadow is not None:
            L.call('cc_to_bf16', L.ptr(self.params), L.ptr(self.shadow), self.layout.total, L.stream_ptr())
        if getattr(self, 'targs', None) is not None:
            self.transpose_tower()

    def set_epoch_permutation(self, perm):
        """Upload one epoch's cube order (generator.py:63-72) and reset the batch counter."""
        self.set_epoch_permutations(np.asarray(perm)[None, :])

    def set_epoch_permutations(self, perms):
        """Upload E epoch orders [E, C] (reset_indices / on_epoch_end, generator.py:63-72); epochs
        cycle through them.  Batch and epoch counters live on the device (state[1], state[2]) and
        are advanced by cc_state_advance, so a step has no host round trip and replays as a graph."""
        p = torch.as_tensor(np.ascontiguousarray(perms, np.int32))
        assert p.shape[1] == self.data.C
        if self.perms is None or self.perms.shape != p.shape:
            self.perms = torch.empty(p.shape, device=self.dev, dtype=torch.int32)
        self.perms.copy_(p)
        self.state[1:3].zero_()
        self.noise_ready = False   # a prefetched batch was drawn from the old order

    def load_batch(self, xs, ys, reg_idx=None):
        """Host-given batch in place of F for the next forward_backward (one process): the rows of
        a Keras batch ``[x_cubes, x_reg], [y_cubes, y_reg]`` as generator.py:38-61,74-103 returns
        them — xs / ys the B noised input / target cubes as card-index lists (or 0/1 rows), reg_idx
        the B regulariser cards (x_reg = their identity rows, y_reg = their M~ rows).  Written into
        the device batch buffers F would fill (x CSR, target bitmask, reg indices, the W1 gradient's
        bit matrix or F's x-row bitmasks), then the step skips F.  Lets the GPU step run on batches
        the reference's own DataGenerator produced (tests/test_gpu_parity_inputs.py)."""
        cfg, V, B = self.cfg, self.cfg.V, self.cfg.batch_size
        if self.dp:
            raise ValueError('load_batch: one process only (each rank draws its own slots)')
        if len(xs) != B or len(ys) != B:
            raise ValueError(f'load_batch: {len(xs)} x rows / {len(ys)} y rows, batch_size is {B}')

        def ids(row):
            a = np.asarray(row)
            if a.ndim == 1 and a.shape[0] == V and V > 2 and a.size and a.min() >= 0 and a.max() <= 1:
                a = np.nonzero(a)[0]            # a dense 0/1 row (an index list of length V holds 2..V-1)
            a = np.unique(a.astype(np.int64))
            if a.size and (a[0] < 0 or a[-1] >= V):
                raise ValueError('load_batch: card index out of range')
            return a
        rows = [ids(r) for r in xs]
        if self.use_reg and not self.full_reg:
            if reg_idx is None or len(reg_idx) != B:
                raise ValueError('load_batch: reg > 0 needs the B regulariser cards')
            reg = np.asarray(reg_idx, np.int64)
            if reg.min() < 0 or reg.max() >= V:
                raise ValueError('load_batch: regulariser card out of range')
            rows += [np.array([j]) for j in reg]
        nrow = len(rows)                         # full mode: its identity rows stay as they are
        if max(len(r) for r in rows) > self.x_cap:
            raise ValueError(f'load_batch: a row holds more than x_cap = {self.x_cap} cards')
        VW = (V + 31) // 32
        cnt = np.zeros(nrow, np.int32)
        idx = np.zeros((nrow, self.x_cap), np.int32)
        xb = np.zeros((nrow, VW * 32), np.uint8)
        for r, a in enumerate(rows):
            cnt[r] = len(a)
            idx[r, :len(a)] = a
            xb[r, a] = 1
        yb = np.zeros((B, VW * 32), np.uint8)
        for b, row in enumerate(ys):
            yb[b, ids(row)] = 1

        def words(bits):   # bit k of word w = column 32 w + k (little-endian bit order)
            return np.packbits(bits, axis=-1, bitorder='little').view(np.int32)
        dev = self.dev
        self.x_cnt[:nrow].copy_(torch.from_numpy(cnt).to(dev))
        self.x_idx[:nrow].copy_(torch.from_numpy(idx).to(dev))
        self.y_bits.copy_(torch.from_numpy(words(yb)).to(dev))
        if self.use_reg and not self.full_reg:
            self.reg_idx[:B].copy_(torch.from_numpy(reg.astype(np.int32)).to(dev))
        if self.x_bits is not None:   # F's x-row bitmasks: the gather / tower launch transposes them
            self.x_bits[:nrow].copy_(torch.from_numpy(words(xb)).to(dev))
        else:                          # the W1 gradient's bit matrix [V][rows/32] directly
            XR = self.xt_rows
            xt = np.zeros((V, (XR + 31) // 32 * 32), np.uint8)
            for r, a in enumerate(rows[:XR]):   # (full mode: the cubes only, XR = B)
                xt[a, r] = 1
            self.xt_bits.copy_(torch.from_numpy(words(xt)).to(dev))
        self.flush()                   # (the previous step's deferred counters / transposes)
        self.noise_ready = True        # forward_backward consumes these buffers, no F
        self.host_batch = True         # step(): eager forward_backward (the graphs hold F)

    def _noise_args(self):
        cfg, V, B = self.cfg, self.cfg.V, self.cfg.batch_size
        return L.NoiseArgs(V=V, B=B, x_cap=self.x_cap, with_reg=int(self.use_reg and not (self.owner or self.full_reg)),
                           seed=cfg.seed,
                           slot_base=cfg.rank * B, batch_stride=B * cfg.world, batch_offset=cfg.rank * B,
                           noise_mean=cfg.noise, noise_std=cfg.noise_std,
                           cube_ptr=self.data.cube_ptr.data_ptr(), cube_idx=self.data.cube_idx.data_ptr(),
                           num_perms=self.perms.shape[0], num_cubes=self.data.C,
                           perm=self.perms.data_ptr(), cdf=self.data.cdf.data_ptr(),
                           neg_sampler=self.data.neg_sampler.data_ptr(), guide=self.data.guide.data_ptr(),
                           guide_log2=self.data.guide_log2, state=self.state.data_ptr(),
                           x_cnt=self.x_cnt.data_ptr(), x_idx=self.x_idx.data_ptr(),
                           y_bits=self.y_bits.data_ptr(),
                           xt_bits=0 if getattr(self, 'xt_in_gather', False) else self.xt_bits.data_ptr(),
                           reg_idx=self.reg_idx.data_ptr(), status=self.status.data_ptr(),
                           xt_rows=self.xt_rows, reg_slots=B * cfg.world, reg_lo=self.reg_rows[0],
                           reg_hi=self.reg_rows[1], reg_cap=self.Breg,
                           x_bits=self.x_bits.data_ptr() if getattr(self, 'xt_in_gather', False) else 0)

    def _gemm(self, M, N, K, A, lda, B, ldb, ta=0, tb=0, epi=L.CC_EPI_STORE, ldc=None, bias=None,
              relu=0, C=None, Cf=None, H=None, y_bits=None, scale=0.0, partials=None, splits=1,
              colsum=None, Ct=None, ldct=0, stream=None, loss_out=None, loss_scale=0.0, ticket=None,
              launch=True, dtype=None, a_scale=None, b_scale=None):
        g = L.GemmArgs(dtype=self.dtype if dtype is None else dtype, ta=ta, tb=tb, epilogue=epi, M=M, N=N,
                       K=K, lda=lda, ldb=ldb, ldc=ldc if ldc is not None else N, splits=splits, relu=relu,
                       A=A, B=B, bias=bias, C=C, Cf=Cf, H=H, y_bits=y_bits, scale=scale,
                       loss_partials=partials, colsum=colsum, Ct=Ct, ldct=ldct,
                       loss_out=loss_out, loss_scale=loss_scale, ticket=ticket,
                       a_scale=a_scale, b_scale=b_scale)
        if launch:
            L.call('cc_gemm', L.C.byref(g), stream if stream is not None else self._s)
        return g

    def _dense_fwd(self, X, rows, K, N, name, out):
        """out[rows] = relu(X[rows] @ W + b) (model.py Dense(relu))."""
        r0, r1 = rows
        self._gemm(r1 - r0, N, K, L.ptr(X[r0:]), K, self.w(name + '/kernel'), N,
                   bias=self.pf(name + '/bias'), relu=1, C=L.ptr(out[r0:]))

    def _dense_bwd(self, Xin, gOut, rows, K, N, name, gIn=None, gIn_f32=None, mask=None):
        """dW = Xin^T gOut with db = colsum(gOut) fused; gIn = (gOut W^T) * [mask > 0]."""
        r0, r1 = rows
        R = r1 - r0
        S = self.tsplits * (R // self.cfg.batch_size)
        if S > 1:   # K = R rows: split-K for parallelism, partials summed in split order
            self._gemm(K, N, R, L.ptr(Xin[r0:]), K, L.ptr(gOut[r0:]), N, ta=1, tb=0,
                       epi=L.CC_EPI_SPLITK, Cf=L.ptr(self.split_buf), splits=S, colsum=L.ptr(self.cs_buf))
            L.call('cc_splitk_reduce', self.dtype, L.ptr(self.split_buf), S, K, N, None, None,
                   self.gp(name + '/kernel'), L.ptr(self.cs_buf), self.gp(name + '/bias'), self._s)
        else:
            self._gemm(K, N, R, L.ptr(Xin[r0:]), K, L.ptr(gOut[r0:]), N, ta=1, tb=0,
                       Cf=self.gp(name + '/kernel'), colsum=self.gp(name + '/bias'))
        if gIn is not None or gIn_f32 is not None:
            self._gemm(R, K, N, L.ptr(gOut[r0:]), N, self.w(name + '/kernel'), N, ta=0, tb=1,
                       epi=L.CC_EPI_MASK, H=L.ptr(mask[r0:]),
                       C=L.ptr(gIn[r0:]) if gIn is not None else None,
                       Cf=L.ptr(gIn_f32[r0:]) if gIn_f32 is not None else None)

    # ------------------------------------------------------------------ the step
    def forward_backward(self, stream=None):
        """One step's gradients into self.grads (no optimizer): F, E, D1/D2 + losses, backward."""
        self.flush(stream, defer=self.noise_ready)   # (F drawn already: nothing reads the counters before E1)
        self.forward_backward_a(stream)
        self.forward_backward_b(stream)

    def forward_backward_a(self, stream=None):
        """F, E, towers forward, both output layers with their losses and weight/input gradients.
        After it the output-layer gradient bucket is final (zero.py overlaps its reduction
        with forward_backward_b)."""
        cfg, lay = self.cfg, self.layout
        V, d, B, R = cfg.V, cfg.d, cfg.batch_size, self.R
        self._s = L.stream_ptr(stream)
        s = self._s
        # ---- F: noise + reg rows (generator.py:38-103); xt_bits arrives zeroed (the previous
        # step's cc_embed_scatter_bwd consumes it)
        if self.noise_ready:       # drawn by the previous step's Adam launch (cc_adam_noise) or
            self.noise_ready = False   # written by load_batch()
            self.host_batch = False
        else:
            na = self._noise_args()
            t = self._tick('cc_noise_fwd')
            L.call('cc_noise_fwd', L.C.byref(na), s)
            t()
        if self.owner:             # the rank's owned rows of the step's global reg draws
            L.call('cc_reg_rows', L.C.byref(self._noise_args()), s)
        # ---- E (model.py:35-42) on R rows: gather + 3 Dense
        t = self._tick('cc_embed_gather_fwd')
        wf = self.wpack[0] if self.wpack is not None else None   # warm the tower forward's weights
        L.call('cc_embed_gather_fwd_xt', self.dtype, self.w('encoder/encoded_1/kernel'),
               self.pf('encoder/encoded_1/bias'), V, d, R, L.ptr(self.x_cnt), L.ptr(self.x_idx),
               self.x_cap, L.ptr(self.H1), L.ptr(wf) if wf is not None else None,
               2 * wf.numel() if wf is not None else 0,
               L.ptr(self.state) if self._adv_deferred else None, self.batches_per_epoch,
               L.ptr(self.x_bits) if self.xt_in_gather and not self.xt_in_tower else None,
               L.ptr(self.xt_bits) if self.xt_in_gather and not self.xt_in_tower else None, self.xt_rows, s)
        self._adv_deferred = False
        t()
        branches = self.branches()
        Br = self.Breg
        if self.fused_tower:
            t = self._tick('cc_tower_fwd')
            L.call('cc_tower_fwd', L.C.byref(self.targs), s)
            t()
        else:
            self._dense_fwd(self.H1, (0, R), d, 256, 'encoder/encoded_2', self.H2)
            self._dense_fwd(self.H2, (0, R), 256, 128, 'encoder/encoded_3', self.H3)
            self._dense_fwd(self.H3, (0, R), 128, 64, 'encoder/bottleneck', self.Zl)
            for pre, rows in branches:
                self._dense_fwd(self.Zl, rows, 64, 128, pre + '/decoded_1', self.D1)
                self._dense_fwd(self.D1, rows, 128, 256, pre + '/decoded_2', self.D2)
                self._dense_fwd(self.D2, rows, 256, d, pre + '/decoded_3', self.D3)
        # ---- D1 output + sigmoid + BCE -> dZ (model.py:64,94; train.py:85)
        if self.mx8 and not self.d3q_in_tower:   # MX-FP8 images of D3: rows (forward A) and transposed (dW A, K = rows)
            L.call('cc_quant_mx8', L.CC_BF16, L.ptr(self.D3), R, d, d, 0, L.ptr(self.D3q), d,
                   L.ptr(self.D3qs), None, s)
            L.call('cc_quant_mx8', L.CC_BF16, L.ptr(self.D3), R, d, d, 1, L.ptr(self.D3tq), R,
                   L.ptr(self.D3tqs), None, s)
        self._fire('hook_d1')   # (zero.py: the output layers' deferred all-gather landed)
        t = self._tick('dec_bce_fwd')
        if self.fused_out:     # logits + BCE + dZ + dWo/dbo in one pass (csrc/decout.hip)
            pk = (L.ptr(self.D3p) if self.D3p is not None else None,
                  L.ptr(self.D3tp) if self.D3p is not None else None, None,
                  self.w('decoder/reconstruct/kernel'),   # Wo [d][V]: slices transposed in LDS
                  self.pf('decoder/reconstruct/bias'), B, d, V, L.ptr(self.y_bits))
            tail = (L.ptr(self.dZ1), self.dz1_ld, self.gp('decoder/reconstruct/kernel'),
                    self.gp('decoder/reconstruct/bias'), L.ptr(self.bce_part), L.ptr(self.loss_dev), 1.0 / (B * V),
                    L.ptr(self.tickets), s)
            if self.y_img is not None:   # (the tower forward launch wrote the mask image)
                L.call('cc_dec_bce_dw_img', L.ptr(self.D3), L.ptr(self.D3t), R, *pk, L.ptr(self.y_img), *tail)
            else:
                L.call('cc_dec_bce_dw_ld', L.ptr(self.D3), L.ptr(self.D3t), R, *pk, *tail)
            self._fire('hook_out')     # dWo / dbo of the D1 output layer final
        elif self.mx8_bce_q:   # config 5: the BCE epilogue writes dZ's MX-FP8 images + the bias grad
            g = self._gemm(B, V, d, **self._dec_fwd(0, 0), tb=1,
                           epi=L.CC_EPI_BCE, bias=self.pf('decoder/reconstruct/bias'),
                           y_bits=L.ptr(self.y_bits), scale=1.0 / (B * V), partials=L.ptr(self.bce_part),
                           loss_out=L.ptr(self.loss_dev), loss_scale=1.0 / (B * V),
                           ticket=L.ptr(self.tickets), launch=False)
            # + the regulariser branch's logits (independent: the same D3 launch's other rows) as
            # extra blocks of the same launch, filling the CUs the BCE tiles leave idle
            g2 = (self._gemm(self.Breg, V, d, **self._dec_fwd(1, B), tb=1,
                             bias=self.pf('decoder_for_reg/reconstruct/bias'), Cf=L.ptr(self.Z2), launch=False)
                  if self.reg_logits_paired else None)
            L.call('cc_gemm_mx8_bce_q2', L.C.byref(g), L.ptr(self.dZq), self.Vp, L.ptr(self.dZqs),
                   L.ptr(self.dZtq[0]), B, L.ptr(self.dZtqs[0]), self.gp('decoder/reconstruct/bias'),
                   L.C.byref(g2) if g2 is not None else None, s)
        elif self.fused_tower:   # Wo^T [V][d]: k-contiguous B operand; also writes dZ^T [V][B]
            self._gemm(B, V, d, **self._dec_fwd(0, 0), tb=1,
                       epi=L.CC_EPI_BCE, bias=self.pf('decoder/reconstruct/bias'), C=L.ptr(self.dZout),
                       y_bits=L.ptr(self.y_bits), scale=1.0 / (B * V), partials=L.ptr(self.bce_part),
                       Ct=L.ptr(self.dZt[0]), ldct=B, loss_out=L.ptr(self.loss_dev),
                       loss_scale=1.0 / (B * V), ticket=L.ptr(self.tickets))
        else:
            self._gemm(B, V, d, L.ptr(self.D3), d, self.w('decoder/reconstruct/kernel'), V,
                       epi=L.CC_EPI_BCE, bias=self.pf('decoder/reconstruct/bias'), C=L.ptr(self.dZout),
                       y_bits=L.ptr(self.y_bits), scale=1.0 / (B * V), partials=L.ptr(self.bce_part),
                       loss_out=L.ptr(self.loss_dev), loss_scale=1.0 / (B * V),
                       ticket=L.ptr(self.tickets))
        t()
        ss = self._fork()          # off the critical path: loss reductions, output-layer dW
        # ---- D2 output + softmax + KL vs M~ rows (model.py:98; train.py:85)
        if self.use_reg and self.fused_reg:   # logits -> softmax -> KL -> dZ, dWo, dbo (decreg.hip)
            lo, hi = self.reg_rows
            t = self._tick("dec_softmax_kl")
            ka = L.DecKlArgs(d=d, V=V, rows=Br, ldt=R, row0=B, D3p=L.ptr(self.D3p), D3tp=L.ptr(self.D3tp),
                             Wo=self.w('decoder_for_reg/reconstruct/kernel'),
                             bo=self.pf('decoder_for_reg/reconstruct/bias'),
                             Mt=self.data.y_reg.data_ptr() - lo * V * 4, tsum=self.tsum.data_ptr() - lo * 8,
                             mt_bytes=hi * V * 4, mt_lo=lo, reg_idx=L.ptr(self.reg_idx),
                             scale=float(self.kl_row_scale), dZ=L.ptr(self.dZout[B:]),
                             gW=self.gp('decoder_for_reg/reconstruct/kernel'),
                             gb=self.gp('decoder_for_reg/reconstruct/bias'), loss_partials=L.ptr(self.kl_part),
                             loss_out=L.ptr(self.loss_dev[1:]), loss_scale=float(self.kl_loss_scale),
                             ticket=L.ptr(self.tickets[1:]), ws=L.ptr(self.kl_ws), flags=self.kl_flags)
            L.call('cc_dec_softmax_kl_dw', L.C.byref(ka), s)
            t()
        elif self.use_reg:
            if self.reg_logits_paired:
                pass   # in the BCE product's launch above
            elif self.fused_tower:
                self._gemm(Br, V, d, **self._dec_fwd(1, B), tb=1,
                           bias=self.pf('decoder_for_reg/reconstruct/bias'), Cf=L.ptr(self.Z2))
            else:
                self._gemm(Br, V, d, L.ptr(self.D3[B:]), d, self.w('decoder_for_reg/reconstruct/kernel'), V,
                           bias=self.pf('decoder_for_reg/reconstruct/bias'), Cf=L.ptr(self.Z2))
            t = self._tick('dec_softmax_kl')
            # M~ row shard [lo, hi): the kernel indexes y_reg[reg_idx * V], so pass the base of
            # row 0 (reg_idx lies in [lo, hi) or is -1 for a masked padding row)
            y_base = L.C.c_void_p(self.data.y_reg.data_ptr() - self.reg_rows[0] * V * 4)
            if self.mx8:   # + dZ's MX-FP8 row image (the dX operand) from the same pass
                L.call('cc_dec_softmax_kl_q', L.ptr(self.Z2), Br, V, y_base, L.ptr(self.reg_idx),
                       float(self.kl_row_scale), L.ptr(self.dZout[B:]), L.ptr(self.kl_part),
                       L.ptr(self.dZq[B:]), self.Vp, L.ptr(self.dZqs[B:]), s)
            else:
                L.call('cc_dec_softmax_kl_fused', self.dtype, L.ptr(self.Z2), Br, V, y_base,
                       L.ptr(self.reg_idx), float(self.kl_row_scale), L.ptr(self.dZout[B:]),
                       L.ptr(self.kl_part), s)
            t()
            if self.fused_tower:   # dZ2^T [V][Breg]: the k-contiguous operand of the reg branch's dW
                L.call('cc_transpose', self.dtype, L.ptr(self.dZout[B:]), Br, V, L.ptr(self.dZt[1]), s)
            ss = self._fork()
            L.call('cc_reduce_loss', L.ptr(self.kl_part), Br, self.kl_loss_scale, L.ptr(self.loss_dev[1:]), ss)
        if self.acc_counts is not None:
            self._metrics_step(s)
        # ---- backward through the output layers and decoder towers.  The output layers' dW
        # (side stream) and dX -> towers (this stream) only share read-only inputs.
        for k, (pre, (r0, r1)) in enumerate(branches):
            if k == 1:                 # branch 0 (D1) done: its dW final, its Wo shadow read
                if self.hook_out is not None and (not self.early_reg_out or self.fused_reg):
                    self._join()       # (dW may have been issued on the side stream)
                    self._fire('hook_out')   # (fused D2: the regulariser's output layer is final too)
                if not self.early_reg_out:
                    self._fire('hook_dx')
            dz = self.dZout[r0:]
            nr = r1 - r0
            splits = self.splits if k == 0 else self.splits_reg
            if self.fused_tower:
                if self.mx8 and k == 0 and not self.mx8_bce_q:   # MX-FP8 dZ (dX A, K = V); the reg branch's
                    # comes out of cc_dec_softmax_kl_q
                    L.call('cc_quant_mx8', L.CC_BF16, L.ptr(dz), nr, V, V, 0, L.ptr(self.dZq[r0:]), self.Vp,
                           L.ptr(self.dZqs[r0:]), None, s)
                if self.mx8 and not (k == 0 and self.mx8_bce_q):   # MX-FP8 dZ^T (dW B, K = rows) + the bias grad
                    L.call('cc_quant_mx8', L.CC_BF16, L.ptr(self.dZt[k]), V, nr, nr, 0, L.ptr(self.dZtq[k]), nr,
                           L.ptr(self.dZtqs[k]), self.gp(pre + '/reconstruct/bias'), s)
                gx = self._gemm(nr, d, self.Vp if self.mx8 else V, **self._dec_dx(k, r0, pre), ta=0, tb=1,
                                epi=L.CC_EPI_SPLITK, Cf=L.ptr(self.split_buf), splits=splits,
                                launch=False)
                if k == 1 and self.fused_reg:   # dWo/dbo came out of cc_dec_softmax_kl_dw: dX only
                    self._dx(gx, r0, nr, splits, pre, s, k=1)
                    L.call('cc_splitk_reduce', self.dtype, L.ptr(self.split_buf), splits, nr, d,
                           L.ptr(self.D3[r0:]), L.ptr(self.gD3[r0:]), None, None, None, s)
                    continue
                if k == 0 and self.fused_out:   # dWo/dbo came out of cc_dec_bce_dw: dX only
                    t = self._tick('dec_dX')
                    self._dx(gx, r0, nr, splits, pre, s)
                    t()
                    wb = self.wpack[1] if self.wpack is not None else None   # warm the tower bwd's weights
                    L.call('cc_splitk_reduce_warm', self.dtype, L.ptr(self.split_buf), splits, nr, d,
                           L.ptr(self.D3[r0:]), L.ptr(self.gD3[r0:]), None, None, None,
                           L.ptr(wb) if wb is not None else None, 2 * wb.numel() if wb is not None else 0, s)
                    continue
                gw = self._gemm(d, V, nr, **self._dec_dw(k, r0), ta=0, tb=1,
                                Cf=self.gp(pre + '/reconstruct/kernel'),
                                colsum=None if self.mx8 else self.gp(pre + '/reconstruct/bias'), launch=False)
                if not self.timing and not self.overlap:   # dX (split-K) and dW in one grouped launch
                    L.call('cc_gemm_pair', L.C.byref(gx), L.C.byref(gw), s)
                else:
                    t = self._tick('dec_dW', self.side if self.overlap else None)
                    L.call('cc_gemm', L.C.byref(gw), ss)
                    t()
                    t = self._tick('dec_dX')
                    L.call('cc_gemm', L.C.byref(gx), s)
                    t()
                L.call('cc_splitk_reduce', self.dtype, L.ptr(self.split_buf), splits, nr, d,
                       L.ptr(self.D3[r0:]), L.ptr(self.gD3[r0:]), None, None, None, s)
                continue
            t = self._tick('dec_dW', self.side if self.overlap else None)
            self._gemm(d, V, nr, L.ptr(self.D3[r0:]), d, L.ptr(dz), V, ta=1, tb=0,
                       Cf=self.gp(pre + '/reconstruct/kernel'), colsum=self.gp(pre + '/reconstruct/bias'),
                       stream=ss)
            t()
            t = self._tick('dec_dX')
            self._gemm(nr, d, V, L.ptr(dz), V, self.w(pre + '/reconstruct/kernel'), V, ta=0, tb=1,
                       epi=L.CC_EPI_SPLITK, Cf=L.ptr(self.split_buf), splits=splits)
            t()
            L.call('cc_splitk_reduce', self.dtype, L.ptr(self.split_buf), splits, nr, d,
                   L.ptr(self.D3[r0:]), L.ptr(self.gD3[r0:]), None, None, None, s)
            rows = (r0, r1)
            self._dense_bwd(self.D2, self.gD3, rows, 256, d, pre + '/decoded_3', gIn=self.gD2, mask=self.D2)
            self._dense_bwd(self.D1, self.gD2, rows, 128, 256, pre + '/decoded_2', gIn=self.gD1, mask=self.D1)
            self._dense_bwd(self.Zl, self.gD1, rows, 64, 128, pre + '/decoded_1', gIn=self.gZl, mask=self.Zl)
        self._join()               # (the side stream's output-layer work before the bucket's exchange)
        self._fire('hook_out')
        self._fire('hook_dx')

    def _fire(self, name):
        f = getattr(self, name)
        if f is not None:
            setattr(self, name, None)
            f()

    def _fire_bucket(self, name):
        f = self.bucket_hooks.pop(name, None)
        if f is not None:
            f()

    def bucket_hook_names(self):
        """Gradient buckets forward_backward_b finalises one by one and fires a hook for (zero.py
        starts each one's exchange there): W1's row chunks (the last with the towers)."""
        if not self.layout.group_biases:
            return ()
        return tuple(f'w1_{i}' for i in range(len(self.layout.w1_chunks)))

    def f_bucket_name(self):
        """The bucket whose sharded Adam launch also draws the next step's F (its update waits for
        the end of backward, as F must): the last W1 chunk, or the towers + E1 bucket."""
        if self.layout.group_biases:
            return f'w1_{len(self.layout.w1_chunks) - 1}'
        return 'towers_e1'

    def _dx(self, gx, r0, nr, splits, pre, s, k=0):
        """Decoder dX split-K partials into split_buf: the LDS-DMA pipelined kernel (dxgemm.hip)
        on the bf16 shapes it takes (the full-mode regulariser's with Wo's fragment image), else
        cc_gemm's register-staged NT path (same partials)."""
        d, V = self.cfg.d, self.cfg.V
        A, lda = self._dz_of(r0)
        if k == 1 and self.WoP is not None and nr % 128 == 0 and dx_splitk_fits(nr, V, d):
            L.call('cc_gemm_dx_splitk_pk', L.ptr(A), lda, L.ptr(self.WoP), nr, d, V, splits,
                   L.ptr(self.split_buf), s)
        elif (self.dx_glds and not self.mx8 and nr % 128 == 0 and d % 128 == 0 and V % 8 == 0
                and dx_splitk_fits(nr, V, d)):
            L.call('cc_gemm_dx_splitk', L.ptr(A), lda, self.w(pre + '/reconstruct/kernel'), V,
                   nr, d, V, splits, L.ptr(self.split_buf), s)
        else:
            L.call('cc_gemm', L.C.byref(gx), s)

    # operands of the decoder output-layer products (branch k, rows [r0, r0 + B)): bf16 NT images
    # (D3, Wo^T, dZ, Wo, D3^T, dZ^T) or their MX-FP8 codes + E8M0 scales
    def _dec_fwd(self, k, r0):
        d = self.cfg.d
        if self.mx8:
            return dict(A=L.ptr(self.D3q[r0:]), lda=d, B=L.ptr(self.WoT8[k]), ldb=d, dtype=L.CC_MX8,
                        a_scale=L.ptr(self.D3qs[r0:]), b_scale=L.ptr(self.WoT8s[k]))
        return dict(A=L.ptr(self.D3[r0:]), lda=d, B=L.ptr(self.WoT[k]), ldb=d)

    def _dec_dx(self, k, r0, pre):
        V = self.cfg.V
        if self.mx8:
            return dict(A=L.ptr(self.dZq[r0:]), lda=self.Vp, B=L.ptr(self.Wo8[k]), ldb=self.Vp,
                        dtype=L.CC_MX8, a_scale=L.ptr(self.dZqs[r0:]), b_scale=L.ptr(self.Wo8s[k]))
        A, lda = self._dz_of(r0)
        return dict(A=L.ptr(A), lda=lda, B=self.w(pre + '/reconstruct/kernel'), ldb=V)

    def _dz_of(self, r0):
        """dZ of the branch starting at row r0 and its row pitch (the fused D1 kernel's own buffer)."""
        if r0 == 0 and self.dZ1 is not None:
            return self.dZ1, self.dz1_ld
        return self.dZout[r0:], self.cfg.V

    def _dec_dw(self, k, r0):
        R, nr = self.R, self.branch_rows()[k]
        if self.mx8:
            return dict(A=L.ptr(self.D3tq[:, r0:]), lda=R, B=L.ptr(self.dZtq[k]), ldb=nr, dtype=L.CC_MX8,
                        a_scale=L.ptr(self.D3tqs[:, r0 // 32:]), b_scale=L.ptr(self.dZtqs[k]))
        return dict(A=L.ptr(self.D3t[:, r0:]), lda=R, B=L.ptr(self.dZt[k]), ldb=nr)

    def _metrics_step(self, s):
        """Keras metrics=['accuracy'] of this step (train.py:87): both outputs' logits recomputed from
        the operands the step used (D3 and the output layers' bf16 / fp32 weights) into fp32, then
        both outputs' categorical accuracy — TF 2.5 picks binary_accuracy only for a last dim of 1
        (compile_utils._get_metric_object) — output 1's against the noised target rows, output 2's
        against the M~ rows' argmax (metrics.hip).  Off the training arithmetic."""
        cfg, V, d, B = self.cfg, self.cfg.V, self.cfg.d, self.cfg.batch_size
        self._gemm(B, V, d, L.ptr(self.D3), d, self.w('decoder/reconstruct/kernel'), V,
                   bias=self.pf('decoder/reconstruct/bias'), Cf=L.ptr(self.Z1m), stream=s)
        L.call('cc_sigmoid_cat_accuracy', L.ptr(self.Z1m), V, L.ptr(self.y_bits), B, V, L.ptr(self.acc_counts), s)
        if self.use_reg:
            ch = self.Z2m.shape[0]
            for r0 in range(0, self.Breg, ch):
                nr = min(ch, self.Breg - r0)
                self._gemm(nr, V, d, L.ptr(self.D3[B + r0:]), d, self.w('decoder_for_reg/reconstruct/kernel'), V,
                           bias=self.pf('decoder_for_reg/reconstruct/bias'), Cf=L.ptr(self.Z2m), stream=s)
                L.call('cc_cat_accuracy', L.ptr(self.Z2m), V, nr, V, L.ptr(self.reg_idx[r0:]), L.ptr(self.t_argmax),
                       self.reg_rows[0], L.ptr(self.acc_counts[1:]), s)

    def take_metrics(self, steps):
        """{'output_1_accuracy', ['output_2_accuracy']} over the steps since the last call (Keras'
        per-epoch Mean of binary / categorical accuracy) and reset the device counts.  Data
        parallel: the counts are summed over the ranks first."""
        c = self.acc_counts.clone()
        self.acc_counts.zero_()
        if self.dp:
            torch.distributed.all_reduce(c)
        c = c.cpu().numpy()
        n1 = float(steps) * self.cfg.batch_size * self.cfg.world   # rows (categorical accuracy)
        out = {'output_1_accuracy': float(c[0]) / n1}
        if self.use_reg:
            out['output_2_accuracy'] = float(c[1]) / max(float(c[2]), 1.0)
        return out

    def forward_backward_b(self, stream=None):
        """Towers backward (both branches' rows together through the shared encoder) and the E1
        row-gather backward."""
        cfg, V, d, R = self.cfg, self.cfg.V, self.cfg.d, self.R
        self._s = L.stream_ptr(stream)
        s = self._s
        if self.fused_tower:
            t = self._tick('cc_tower_bwd')
            if self.f_in_tower:              # + F of the next step (+ the output layers' Adam tails)
                rg = list(self.wo_ranges or []) + [(0, 0), (0, 0)]
                (a0, b0), (a1, b1) = rg[0], rg[1]
                L.call('cc_tower_bwd_chain_noise', L.C.byref(self.targs), L.C.byref(self._noise_args()),
                       self.batches_per_epoch, L.ptr(self.params), L.ptr(self.m), L.ptr(self.v), L.ptr(self.grads),
                       L.ptr(self.shadow), a0, b0 - a0, a1, b1 - a1, L.ptr(self.state), cfg.lr, cfg.beta1,
                       cfg.beta2, cfg.eps, s)
            elif self.wo_ranges is not None:   # + TF Adam on the output layers' tails beside the chains
                (a0, b0), (a1, b1) = self.wo_ranges[0], (self.wo_ranges + [(0, 0)])[1]
                L.call('cc_tower_bwd_chain_adam', L.C.byref(self.targs), L.ptr(self.params), L.ptr(self.m),
                       L.ptr(self.v), L.ptr(self.grads), L.ptr(self.shadow), a0, b0 - a0, a1, b1 - a1,
                       L.ptr(self.state), cfg.lr, cfg.beta1, cfg.beta2, cfg.eps, s)
            else:
                L.call('cc_tower_bwd_chain', L.C.byref(self.targs), s)
            t()
            ss = self._fork()      # per-block dW slabs + their reduce overlap the E1 scatter
            # direct dW: from the packed images (any row count) or LDS-staged (rows <= ~1184)
            direct = self.hpt is not None or max(R, cfg.batch_size) <= 1184
            if self.dtype == L.CC_BF16 and direct:
                L.call('cc_tower_bwd_dw_direct', L.C.byref(self.targs), ss)
            else:
                L.call('cc_tower_bwd_dw', L.C.byref(self.targs), ss)
                L.call('cc_tower_reduce', L.C.byref(self.targs), ss)
        else:
            self._dense_bwd(self.H3, self.gZl, (0, R), 128, 64, 'encoder/bottleneck', gIn=self.gH3, mask=self.H3)
            self._dense_bwd(self.H2, self.gH3, (0, R), 256, 128, 'encoder/encoded_3', gIn=self.gH2, mask=self.H2)
            self._dense_bwd(self.H1, self.gH2, (0, R), d, 256, 'encoder/encoded_2', gIn_f32=self.gPre1, mask=self.H1)
        t = self._tick('cc_embed_scatter_bwd')
        XR = self.xt_rows          # rows in the bitmask product (full mode: the cubes only)
        chunks = self.layout.w1_chunks if self.layout.group_biases else [(0, V)]
        if self.eg_tickets is not None and self.fuse_w1:   # column slices + TF Adam on W1 in the epilogue
            cfg_ = self.cfg
            src, pk = (self.gpre1p, 1) if self.gpre1p is not None else (self.gPre1T, 0)
            if self.reg_by_index:   # + the reg rows by index (rows B .. of the dPre1 image)
                L.call('cc_embed_grad_cs_adam_reg', L.ptr(src), pk, V, d, XR, self.RP, L.ptr(self.xt_bits),
                       self.gp('encoder/encoded_1/bias'), self._eg_tk(), L.ptr(self.params), L.ptr(self.m),
                       L.ptr(self.v), L.ptr(self.shadow), L.ptr(self.state), cfg_.lr, cfg_.beta1, cfg_.beta2,
                       cfg_.eps, L.ptr(self.reg_idx), self.Breg, cfg.batch_size // 16, s)
            else:
                L.call('cc_embed_grad_cs_adam', L.ptr(src), pk, V, d, XR, self.RP, L.ptr(self.xt_bits),
                       self.gp('encoder/encoded_1/bias'), self._eg_tk(), L.ptr(self.params), L.ptr(self.m),
                       L.ptr(self.v), L.ptr(self.shadow), L.ptr(self.state), cfg_.lr, cfg_.beta1, cfg_.beta2,
                       cfg_.eps, s)
        elif self.eg_tickets is not None:   # column slices (cc_embed_grad_cs), from the packed image or dPre1^T
            src, pk = (self.gpre1p, 1) if self.gpre1p is not None else (self.gPre1T, 0)
            # data parallel: W1's row chunks one launch each (the bias row with the last), each
            # chunk's exchange starting as soon as its launch is issued (zero.py bucket hooks);
            # every W1 tile is computed as in the one-launch product (bit-identical)
            gw, gb = self.layout.offset('encoder/encoded_1/kernel'), self.gp('encoder/encoded_1/bias')
            for i, (r0, r1) in enumerate(chunks):
                gbi = gb if i == len(chunks) - 1 else None
                if self.reg_by_index:
                    L.call('cc_embed_grad_cs_reg', L.ptr(src), pk, r1 - r0, d, XR, self.RP, L.ptr(self.xt_bits[r0:]),
                           L.ptr(self.grads[gw + r0 * d:]), gbi, self._eg_tk(), L.ptr(self.reg_idx), self.Breg,
                           cfg.batch_size // 16, r0, s)
                else:
                    L.call('cc_embed_grad_cs', L.ptr(src), pk, r1 - r0, d, XR, self.RP, L.ptr(self.xt_bits[r0:]),
                           L.ptr(self.grads[gw + r0 * d:]), gbi, self._eg_tk(), s)
                if i + 1 < len(chunks):
                    self._fire_bucket(f'w1_{i}')
        elif self.gpre1p is not None:
            L.call('cc_embed_grad_packed', L.ptr(self.gpre1p), V, d, XR, self.RP, L.ptr(self.xt_bits),
                   self.gp('encoder/encoded_1/kernel'), self.gp('encoder/encoded_1/bias'), s)
        elif self.embed_mfma:
            L.call('cc_embed_grad_mfma', L.ptr(self.gPre1T), V, d, XR, self.RP, L.ptr(self.xt_bits),
                   self.gp('encoder/encoded_1/kernel'), self.gp('encoder/encoded_1/bias'), s)
        else:
            L.call('cc_embed_scatter_bwd', L.ptr(self.gPre1), V, d, XR, L.ptr(self.xt_bits),
                   self.gp('encoder/encoded_1/kernel'), self.gp('encoder/encoded_1/bias'), s)
        if self.full_reg:          # identity rows: dW1[lo + r] += dPre1[B + r]
            B = cfg.batch_size
            L.call('cc_embed_identity_add', self.dtype, L.ptr(self.gPre1[B:]),
                   self.reg_rows[1] - self.reg_rows[0], d, self.reg_rows[0],
                   self.gp('encoder/encoded_1/kernel'), self.gp('encoder/encoded_1/bias'), L.ptr(self.id_ws), s)
        t()
        if self.fused_tower:       # the towers' dW (side stream) ride in the last W1 chunk's bucket
            self._join()
        for i in range(len(chunks)):   # (the W1 chunks not fired above: the last, or all of them)
            self._fire_bucket(f'w1_{i}')

    def _eg_tk(self):
        """W1-gradient tickets (its last block per row chunk clears the chunk's xt words), or None
        when the next E1 gather rewrites every xt word (xt_in_gather)."""
        return None if self.xt_in_gather else L.ptr(self.eg_tickets)

    def apply_adam(self, stream=None):
        """TF Adam over every trained parameter (+ bf16 shadow refresh)."""
        cfg = self.cfg
        n = self.layout.total if self.use_reg else self.layout.main_total
        t = self._tick('cc_adam_dense')
        if self.prefetch:     # + F for the next step in the same launch
            na = self._noise_args()
            # (f_in_tower: F of the next step is already drawn in the tower backward launch)
            fn = 'cc_adam_pack2' if self.f_in_tower else 'cc_adam_noise_pack2'
            if self.adam_packs and self.rest_ranges is not None:   # the complement of the tower launch's
                o = self.w1_off                                      # ranges (pack offsets count from o)
                (a0, b0), (a1, b1) = self.rest_ranges[0], (self.rest_ranges + [(o, o)])[1]
                L.call(fn, L.ptr(self.params[o:]), L.ptr(self.m[o:]), L.ptr(self.v[o:]),
                       L.ptr(self.grads[o:]), L.ptr(self.shadow[o:]), a0 - o, b0 - a0, a1 - o, b1 - a1,
                       cfg.lr, cfg.beta1, cfg.beta2, cfg.eps, L.C.byref(na), self.batches_per_epoch,
                       L.C.byref(self.adam_pack), L.stream_ptr(stream))
            elif self.adam_packs:   # + packed tower images + step counters
                o = self.w1_off if self.fuse_w1 else 0   # (W1 already updated by its gradient kernel)
                L.call(fn, L.ptr(self.params[o:]), L.ptr(self.m[o:]), L.ptr(self.v[o:]),
                       L.ptr(self.grads[o:]), L.ptr(self.shadow[o:]), 0, n - o, 0, 0, cfg.lr, cfg.beta1,
                       cfg.beta2, cfg.eps, L.C.byref(na), self.batches_per_epoch, L.C.byref(self.adam_pack),
                       L.stream_ptr(stream))
            else:
                L.call('cc_adam_noise', L.ptr(self.params), L.ptr(self.m), L.ptr(self.v),
                       L.ptr(self.grads), L.ptr(self.shadow), n, cfg.lr, cfg.beta1, cfg.beta2, cfg.eps,
                       L.C.byref(na), self.batches_per_epoch, L.stream_ptr(stream))
            self.noise_ready = True
        else:
            L.call('cc_adam_dense', L.ptr(self.params), L.ptr(self.m), L.ptr(self.v), L.ptr(self.grads),
                   L.ptr(self.shadow), n, L.ptr(self.state), cfg.lr, cfg.beta1, cfg.beta2, cfg.eps,
                   L.stream_ptr(stream))
        t()

    def apply_rest(self, stream=None, defer=False):
        """Advance the device step/epoch counters and refresh the transposed operand copies
        (the decoder's Wo^T on the side stream, concurrently)."""
        if self.adam_packs:   # packed tower images already written by the Adam launch
            self.refresh_decoder_operands(L.stream_ptr(stream))
            if defer:         # counters: in the next forward's E1 gather launch
                self._adv_deferred = True
            else:
                L.call('cc_state_advance', L.ptr(self.state), self.batches_per_epoch, L.stream_ptr(stream))
            return
        if self.fused_tower and stream is None:
            ss = self._fork()
            self.refresh_decoder_operands(ss)
            L.call('cc_tower_transpose_advance', L.C.byref(self.targs), L.ptr(self.state),
                   self.batches_per_epoch, L.stream_ptr(None))
            self._join()
            return
        L.call('cc_state_advance', L.ptr(self.state), self.batches_per_epoch, L.stream_ptr(stream))
        self.transpose_tower(stream)

    def apply(self, stream=None):
        self.apply_adam(stream)
        self.apply_rest(stream)

    # ------------------------------------------------------------------ data parallel (zero.py)
    def adam_range(self, lo, n, g, stream=None):
        """TF Adam over [lo, lo+n) of the flat buffers with the gradient slice g (a tensor)."""
        cfg = self.cfg
        L.call('cc_adam_dense', L.ptr(self.params[lo:]), L.ptr(self.m[lo:]), L.ptr(self.v[lo:]),
               L.ptr(g), L.ptr(self.shadow[lo:]) if self.shadow is not None else None, n,
               L.ptr(self.state), cfg.lr, cfg.beta1, cfg.beta2, cfg.eps, L.stream_ptr(stream))

    def refresh_range(self, lo, hi, stream=None):
        if self.shadow is not None:
            L.call('cc_to_bf16', L.ptr(self.params[lo:]), L.ptr(self.shadow[lo:]), hi - lo,
                   L.stream_ptr(stream))

    def adam_noise_range(self, lo, n, g, stream=None):
        """adam_range + F of the NEXT step in the same launch (cc_adam_noise: F's latency-bound blocks
        first, the shard's Adam blocks streaming around them) — data parallel, on the bucket whose
        update starts once this step's backward has released the batch buffers."""
        cfg = self.cfg
        L.call('cc_adam_noise', L.ptr(self.params[lo:]), L.ptr(self.m[lo:]), L.ptr(self.v[lo:]), L.ptr(g),
               L.ptr(self.shadow[lo:]) if self.shadow is not None else None, n, cfg.lr, cfg.beta1,
               cfg.beta2, cfg.eps, L.C.byref(self._noise_args()), self.batches_per_epoch, L.stream_ptr(stream))

    def noise_next(self, stream=None):
        """F of the NEXT step (cc_noise_next: the state advanced as apply_rest will) — data
        parallel: issued after this step's backward, beside the exchange of the last buckets."""
        t = self._tick('cc_noise_fwd')
        L.call('cc_noise_next', L.C.byref(self._noise_args()), self.batches_per_epoch, L.stream_ptr(stream))
        t()

    def _sharded(self):
        if self.sharded is None:
            from .zero import ShardedStep
            self.sharded = ShardedStep(self)
        return self.sharded

    def _dp_call(self, g=None, timing=False):
        """The sharded step (zero.py) over graph replays of its parts (g) or eager launches.  The next
        step's F: inside the towers + E1 bucket's sharded Adam launch (dp_f_in_adam; that bucket's
        update waits for the end of backward, as F must), else its own launch after backward."""
        sh = self._sharded()
        fuse_f = self.prefetch_dp and self.cfg.dp_f_in_adam
        tb = sh.bucket(self.f_bucket_name())['gshard'] if fuse_f else None

        def adam_fn(lo, n, gs):
            if gs is tb:
                self.adam_noise_range(lo, n, gs)
            else:
                self.adam_range(lo, n, gs)
        sh.step(
            phase_a=g[0].replay if g else self.forward_backward_a,
            phase_b=g[1].replay if g else self.forward_backward_b,
            rest=g[2].replay if g else self.apply_rest,
            adam_fn=adam_fn,
            refresh_fn=lambda lo, hi: self.refresh_range(lo, hi),
            timing=timing,
            after_b=self.noise_next if self.prefetch_dp and not fuse_f else None,
            hooks=g is None and sh.comm is not None)
        self.noise_ready = self.prefetch_dp

    def step_dp(self, timing=False, no_comm=False):
        """One data-parallel step: bucketed reduce-scatter overlapped with the towers' backward,
        Adam on this rank's shards, all-gathered parameters (zero.py); the next step's F beside the
        last buckets' exchange.  Steady state over RCCL: one replay of the whole-step graph.
        no_comm: replay the timing reference captured without the collectives (bench.py)."""
        g = self.graphs
        gd = self.g_dp_nocomm if no_comm else self.g_dp
        if gd is not None and not timing and (self.noise_ready or not self.prefetch_dp):
            gd.replay()
            # the replayed step deferred its output-layer all-gather like an eager one: flush() and
            # gather_state() must issue it before anything reads the shadow outside a step
            self.sharded.out_pending = self.sharded.defer_out
            return
        self._dp_call(g, timing)

    def dp_defer_out_ok(self):
        """zero.py may defer the output layers' all-gather to the next step's head: nothing between
        this step's Adam and the next D1 launch reads the output layers' shadow (the decoder kernels
        read Wo straight from it; no Wo^T, MX-FP8 or fragment image is refreshed from it)."""
        return bool(self.cfg.dp_defer_out and self.fused_out and (not self.use_reg or self.fused_reg)
                    and self.WoP is None and not self.mx8)

    def flush(self, stream=None, defer=False):
        """Run the previous step's deferred counters/transposes (before reading state or the
        transposed operands from outside the step) and, data parallel, a deferred output-layer
        all-gather (a collective: every rank calls flush).  defer (forward_backward only): the
        counter advance may ride in the forward's first launch."""
        if getattr(self, 'sharded', None) is not None:
            self.sharded.flush_out()
        if self.pending_rest:
            self.pending_rest = False
            self.apply_rest(stream, defer=defer)

    def run_fb(self, stream=None):
        """Forward/backward of one step (graph replay or eager), preceded by the previous step's
        deferred counters/transposes."""
        if self.graphs is not None:
            g_fb, _, _, g_main, _ = self.graphs
            if self.pending_rest and g_main is not None and (self.noise_ready or not self.prefetch):
                g_main.replay()     # previous step's rest + this forward/backward
            else:
                self.flush()
                if self.noise_ready:   # (captured with F inside; redraw, identically)
                    self.noise_ready = False
                g_fb.replay()
            self.pending_rest = False
            self.noise_ready = False
        else:
            self.forward_backward(stream)

    def run_adam(self, stream=None, events=None):
        """Adam (graph replay, or an eager launch bracketed by `events` = (e0, e1))."""
        if events is not None:   # the Adam kernel alone between the events (an eager launch:
            events[0].record()   # a graph replay there would add its launch edge to the interval)
            self.apply_adam(stream)
            events[1].record()
        elif self.graphs is not None:
            self.graphs[1].replay()
            self.noise_ready = self.prefetch   # (captured with the next step's F in the launch)
        else:
            self.apply_adam(stream)
        self.pending_rest = True

    def _steady(self):
        return (not self.host_batch and self.graphs is not None and self.graphs[4] is not None and self.pending_rest
                and (self.noise_ready or not self.prefetch))

    def step(self, stream=None):
        if self.dp:
            self.step_dp()
            return
        if self.host_batch:            # a load_batch() batch: eager forward/backward, no F
            self.host_batch = False
            self.forward_backward(stream)
            self.run_adam(stream)
            return
        if self._steady():
            self.graphs[4].replay()    # steady state: rest(k-1) + fwd/bwd(k) + Adam(k) in one graph
            self.pending_rest = True
            self.noise_ready = self.prefetch
            return
        self.run_fb(stream)
        self.run_adam(stream)

    def step_many(self, n, loss_acc=None):
        """n steps.  In the one-process steady state, graph_steps of them at a time replay one
        captured graph of graph_steps consecutive whole steps (every step's kernels exactly as
        step() launches them; the device counters advance inside): the ~6-9 us boundary between
        two graph replays is paid once per graph_steps steps.  loss_acc: a [2] fp64 device tensor
        that accumulates every step's (bce, kl) — it must be the tensor capture() was given."""
        while n > 0:
            # the largest captured multi-step graph that fits (graph_steps, then halves of it: a
            # remainder of n replays in log2 graphs, not step by step)
            m = max((k for k in self.g_multi_sizes if k <= n), default=0)
            if (m > 0 and self._steady() and (loss_acc is None) == (self.multi_acc is None)
                    and (loss_acc is None or loss_acc is self.multi_acc)):
                self.g_multi_sizes[m].replay()
                self.pending_rest = True
                self.noise_ready = self.prefetch
                n -= m
                continue
            self.step()
            if loss_acc is not None:
                loss_acc += self.loss_dev
            n -= 1

    def capture(self, loss_acc=None):
        """Capture the step as three hipGraphs (torch.cuda.CUDAGraph over our own kernel launches):
        forward_backward | Adam | counters+transposes (data parallel: forward_backward_a |
        forward_backward_b | counters+transposes, with zero.py's collectives and sharded Adam
        between them).  Every buffer is preallocated and the step/epoch counters are
        device-resident, so replays are exact repeats of the eager step.  bench.py brackets the
        Adam kernel with HIP events to time the step's bytes-dominant kernel in the timed region."""
        timing, self.timing = self.timing, False
        self.flush()
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream())
        saved = self.state.clone()
        # the fused W1 (and Wo) Adam updates them inside forward_backward: undo the warm-up's update
        spans = ([(0, self.w1_off)] if self.fuse_w1 else []) + (list(self.wo_ranges) if self.wo_ranges else [])
        saved_spans = [[b[lo:hi].clone() for b in (self.params, self.m, self.v, self.shadow)] for lo, hi in spans]
        with torch.cuda.stream(s):           # warm-up launch outside capture (lazy module loads)
            self.forward_backward()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for (lo, hi), cs in zip(spans, saved_spans):
            for b, c in zip((self.params, self.m, self.v, self.shadow), cs):
                b[lo:hi].copy_(c)
        g_fb, g_adam, g_rest = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        if self.dp:   # (forward_backward_a | forward_backward_b | counters): the
            self.noise_ready = False           # sharded optimizer's collectives run between them
            with torch.cuda.graph(g_fb):       # (F inside: the first step after a capture)
                self.forward_backward_a()
            with torch.cuda.graph(g_adam):
                self.forward_backward_b()
        else:
            self.noise_ready = False
            with torch.cuda.graph(g_fb):       # F inside
                self.forward_backward()
            with torch.cuda.graph(g_adam):     # (with prefetch: + the next step's F)
                self.apply_adam()
        g_main = g_all = None
        with torch.cuda.graph(g_rest):
            self.apply_rest()
        self.g_dp = self.g_dp_nocomm = None
        if self.dp and self.cfg.dp_graph and self._sharded().nccl:
            self._capture_dp()
        if not self.dp:   # rest of step k + forward/backward of step k+1 (+ its Adam)
            g_main, g_all = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            self.noise_ready = self.prefetch   # F already drawn by step k's Adam launch
            with torch.cuda.graph(g_main):
                self.apply_rest(defer=True)
                self.forward_backward()
            self.noise_ready = self.prefetch
            with torch.cuda.graph(g_all):
                self.apply_rest(defer=True)
                self.forward_backward()
                self.apply_adam()
        self.g_multi, self.multi_n, self.multi_acc, self.g_multi_sizes = None, 0, None, {}
        if not self.dp and self.cfg.graph_steps > 1:   # step_many: graph_steps whole steps (and
            m = self.cfg.graph_steps                    # graphs of its halves, for remainders)
            while m > 1:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(m):
                        self.noise_ready = self.prefetch
                        self.apply_rest(defer=True)
                        self.forward_backward()
                        self.apply_adam()
                        if loss_acc is not None:
                            loss_acc += self.loss_dev
                self.g_multi_sizes[m] = g
                m //= 2
            self.g_multi = self.g_multi_sizes[self.cfg.graph_steps]
            self.multi_n, self.multi_acc = self.cfg.graph_steps, loss_acc
        torch.cuda.synchronize()
        self.state.copy_(saved)
        if loss_acc is not None:
            loss_acc.zero_()
        if self.acc_counts is not None:   # the eager warm-up step above counted its metrics
            self.acc_counts.zero_()
        self.noise_ready = False
        self.graphs = (g_fb, g_adam, g_rest, g_main, g_all)
        self.timing = timing

    def _capture_dp(self):
        """The whole data-parallel step as ONE graph: forward_backward_a, the first bucket's
        reduce-scatter / sharded Adam / all-gather on the comm stream beside forward_backward_b, the
        next step's F beside the later buckets' exchange, then the counters and transposed operands.
        RCCL collectives are captured on the comm stream (it forks from and joins the capturing
        stream); the communicator's lazy set-up runs first (ShardedStep.warm).  Assumes F already
        drawn (noise_ready) — the first step after a capture runs the parts instead.  Also captures
        the same step without the collectives (bench.py's exposed-exchange reference)."""
        sh = self._sharded()
        sh.warm()
        graphs = []
        for no_comm in (False, True):
            g = torch.cuda.CUDAGraph()
            self.noise_ready = self.prefetch_dp
            sh.no_comm = no_comm
            try:
                with torch.cuda.graph(g):
                    self._dp_call(None, False)
            except Exception as e:   # never a silent fallback: the caller picks the parts path itself
                raise RuntimeError(
                    f'capturing the whole data-parallel step (RCCL collectives inside) failed on rank '
                    f'{self.cfg.rank} of {self.cfg.world}: {e!r}; rerun with TrainConfig(dp_graph=False) / '
                    f'bench.py --dp-graph 0 (graph parts with eager collectives)') from e
            finally:
                sh.no_comm = False
            graphs.append(g)
        self.g_dp, self.g_dp_nocomm = graphs

    # ------------------------------------------------------------------ inspection (tests)
    def losses(self, loss_dev=None):
        """{'bce', 'kl', 'loss'} of the last step (or of a given [2] device vector)."""
        l = (self.loss_dev if loss_dev is None else loss_dev).cpu().numpy()
        bce, kl = float(l[0]), float(l[1]) if self.use_reg else 0.0
        return {'bce': bce, 'kl': kl, 'loss': bce + self.cfg.reg * kl}

    def batch_lists(self):
        """The last noised batch as host lists: (x lists (R rows), y lists (B rows), reg idx)."""
        cnt = self.x_cnt.cpu().numpy()
        idx = self.x_idx.cpu().numpy()
        xs = [idx[r, :cnt[r]].copy() for r in range(self.R)]
        yb = self.y_bits.cpu().numpy().view(np.uint32)
        ys = []
        for b in range(self.cfg.batch_size):
            bits = np.unpackbits(yb[b].view(np.uint8), bitorder='little')[:self.cfg.V]
            ys.append(np.nonzero(bits)[0])
        return xs, ys, self.reg_idx.cpu().numpy().copy()

    def params_dict(self):
        return self.layout.unpack(self.params.cpu().numpy())

    # ------------------------------------------------------------------ standard-layout views
    def standard(self, buf):
        """A device flat buffer (params / m / v / grads) in the standard cc_param_layout (numpy)."""
        flat = buf.detach().cpu().numpy()
        return flat if self.layout is self.std_layout else self.std_layout.convert(flat, self.layout)

    def load_standard(self, buf, flat):
        flat = np.asarray(flat, np.float32)
        if self.layout is not self.std_layout:
            flat = self.layout.convert(flat, self.std_layout)
        buf.copy_(torch.as_tensor(flat, dtype=torch.float32))
