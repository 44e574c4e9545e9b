"""DataGenerator — device-resident mirror of ``src/ml/generator.py:DataGenerator``.

Same constructor and Sequence protocol (generator.py:6-15, 32-72):
    DataGenerator(adj_mtx, cubes, batch_size=64, shuffle=True, to_fit=True, noise=0.2, noise_std=0.1)
    len(gen) == C // batch_size           (generator.py:36, remainder dropped)
    gen[i]                                -> [x_cubes, x_reg], [y_cubes, y_reg] (to_fit) or
                                             [x_cubes, x_reg], dense float64 [B, V] like :58-61
    gen.device_batch(i)                   -> the same batch kept in HBM (NoisedBatch)
    gen.on_epoch_end()                    -> reshuffle (generator.py:68-72)
``adj_mtx`` is M~ (train.py:69-71 applied), ``cubes`` a dense 0/1 [C, V] matrix (the reference's
build_cubes output, utils.py:57-73), a list of card-index lists, or a CSR (indptr, indices).

Differences by design: batches never leave HBM (x as a CSR of card ids, y and the
transposed x as bitmasks, reg rows as indices into the resident M~), and the draws come from the
counter-based Philox law of cc_noise_fwd instead of numpy's global MT19937 stream (same
distribution; tests/test_oracle.py checks the two laws agree statistically).
"""
import numpy as np
import torch

from . import _lib as L
from .trainer import DeviceDataset


def _to_csr(cubes):
    if isinstance(cubes, tuple) and len(cubes) == 2:
        return np.asarray(cubes[0], np.int64), np.asarray(cubes[1], np.int32)
    if isinstance(cubes, (list, tuple)):
        lists = [np.unique(np.asarray(c, np.int64)) for c in cubes]
    else:
        a = np.asarray(cubes)
        lists = [np.nonzero(a[c] == 1)[0] for c in range(a.shape[0])]   # generator.py:83
    indptr = np.zeros(len(lists) + 1, np.int64)
    indptr[1:] = np.cumsum([len(l) for l in lists])
    idx = np.concatenate(lists).astype(np.int32) if lists else np.zeros(0, np.int32)
    return indptr, idx


class NoisedBatch:
    """One batch as generate_data (generator.py:74-103) produces it, kept on the device."""

    def __init__(self, x_cnt, x_idx, y_bits, reg_idx, y_reg, V):
        self.x_cnt, self.x_idx, self.y_bits, self.reg_idx, self.y_reg, self.V = x_cnt, x_idx, y_bits, reg_idx, y_reg, V

    def x_lists(self):
        cnt, idx = self.x_cnt.cpu().numpy(), self.x_idx.cpu().numpy()
        return [idx[r, :cnt[r]] for r in range(len(cnt))]

    def y_dense(self):
        yb = self.y_bits.cpu().numpy().view(np.uint32)
        return np.stack([np.unpackbits(r.view(np.uint8), bitorder='little')[:self.V] for r in yb]).astype(np.float64)

    def x_dense(self, rows=None):
        lists = self.x_lists()
        B = len(self.y_bits)
        out = np.zeros((B, self.V))
        for b in range(B):
            out[b, lists[b]] = 1
        return out


class DataGenerator:
    def __init__(self, adj_mtx, cubes, batch_size=64, shuffle=True, to_fit=True, noise=0.2,
                 noise_std=0.1, seed=0, device='cuda', neg_sampler=None):
        self.noise, self.noise_std = noise, noise_std
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.to_fit = to_fit
        self.seed = seed
        indptr, idx = _to_csr(cubes)
        self.N_cubes = len(indptr) - 1
        self.N_cards = (int(adj_mtx.shape[1]) if adj_mtx is not None else
                        len(neg_sampler) if neg_sampler is not None else int(idx.max()) + 1)
        self.data = DeviceDataset(csr=(indptr, idx), num_cards=self.N_cards, y_mtx=adj_mtx,
                                  neg_sampler=neg_sampler, device=device)
        self.neg_sampler = self.data.neg_sampler_host          # generator.py:30
        self._rng = np.random.default_rng(seed)
        self.epoch = 0
        self.reset_indices()
        self._trainer = None

    def __len__(self):
        return self.N_cubes // self.batch_size

    def reset_indices(self):
        self.indices = np.arange(self.N_cubes)
        if self.shuffle:
            self._rng.shuffle(self.indices)

    def on_epoch_end(self):
        self.epoch += 1
        self.reset_indices()

    def epoch_permutations(self, epochs):
        """The next `epochs` epoch orders (for a whole-fit, graph-replayable upload).  Keras calls
        on_epoch_end after every epoch, the last included, so a later fit() starts on a fresh order."""
        perms = []
        for _ in range(epochs):
            perms.append(self.indices.copy())
            self.on_epoch_end()
        return np.stack(perms)

    def __getitem__(self, batch_number):
        """generator.py:38-61: ``[x_cubes, x_reg], [y_cubes, y_reg]`` when to_fit, else
        ``[x_cubes, x_reg]`` — dense float64 [B, V] numpy arrays (x_reg = one-hot rows of the reg
        cards, y_reg = their M~ rows).  F runs on the GPU (cc_noise_fwd); use device_batch() to keep
        the batch in HBM."""
        nb = self.device_batch(batch_number)
        B, V = len(nb.y_bits), self.N_cards
        x_cubes = nb.x_dense()
        reg = nb.reg_idx.cpu().numpy() if self.data.y_reg is not None else None
        x_reg = np.zeros((B, V))
        if reg is not None:
            x_reg[np.arange(B), reg] = 1.0
        if not self.to_fit:
            return [x_cubes, x_reg]
        y_reg = (nb.y_reg.cpu().numpy().astype(np.float64) if nb.y_reg is not None
                 else np.zeros((B, V)))
        return [x_cubes, x_reg], [nb.y_dense(), y_reg]

    def device_batch(self, batch_number):
        """Run F (cc_noise_fwd) for batch `batch_number` of the current epoch; device-resident."""
        from .trainer import TrainConfig, Trainer
        if self._trainer is None:
            cfg = TrainConfig(V=self.N_cards, d=64, batch_size=self.batch_size, reg=1.0 if self.data.y_reg is not None else 0.0,
                              noise=self.noise, noise_std=self.noise_std, seed=self.seed, dtype='fp32')
            self._trainer = Trainer(cfg, self.data)
        tr = self._trainer
        tr.set_epoch_permutation(self.indices)
        tr.state[0] = self.epoch * len(self) + batch_number
        tr.state[1] = batch_number
        tr.xt_bits.zero_()
        na = tr._noise_args()
        L.call('cc_noise_fwd', L.C.byref(na), L.stream_ptr())
        torch.cuda.synchronize()
        y_reg = (self.data.y_reg[tr.reg_idx.long()] if self.data.y_reg is not None else None)
        return NoisedBatch(tr.x_cnt.clone(), tr.x_idx.clone(), tr.y_bits.clone(), tr.reg_idx.clone(),
                           y_reg, self.N_cards)
