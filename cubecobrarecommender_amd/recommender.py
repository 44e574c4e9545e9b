"""Resident-model recommend path: fp32 forward (bit-exact pinned order) + top-N on the GPU.

Replaces the hot part of ``src/scripts/ml_recommend.py:78-108`` and
``web/ml_recommend_web.py:39-64``: ``model.encoder(x)`` -> ``model.decoder(z)`` -> ``argsort``
-> additions / cuts.  Unlike the reference web path (which reloads the ~390 MB SavedModel on every
request, ml_recommend_web.py:37) the weights stay resident in HBM; requests are serialised per
``Recommender`` with a lock (Flask runs threaded, web/__init__.py:41) and run on its own stream.
"""
import threading

import numpy as np
import torch

from . import _lib as L
from .layout import Layout


class Recommender:
    def __init__(self, params_flat, V, d, device='cuda'):
        L.lib()
        self.V, self.d = int(V), int(d)
        self.layout = Layout(V, d)
        self.dev = torch.device(device)
        p = torch.as_tensor(np.asarray(params_flat, np.float32)) if not torch.is_tensor(params_flat) else params_flat
        self.params = p.to(self.dev, torch.float32).contiguous()
        assert self.params.numel() >= self.layout.main_total
        self.stream = torch.cuda.Stream(device=self.dev)
        self.lock = threading.Lock()
        self._alloc(1)
        self.topn_ws = torch.zeros(int(L.lib().cc_topn_workspace_size(V)) // 4 + 1,
                                   device=self.dev, dtype=torch.int32)
        self.additions = torch.zeros(V, device=self.dev, dtype=torch.int32)
        self.add_vals = torch.zeros(V, device=self.dev, dtype=torch.float32)
        self.cut_vals = torch.zeros(V, device=self.dev, dtype=torch.float32)
        self.n_add = torch.zeros(1, device=self.dev, dtype=torch.int32)
        self.order = torch.zeros(V, device=self.dev, dtype=torch.int32)
        self.idx_dev = torch.zeros(V + 2, device=self.dev, dtype=torch.int32)
        self.pin_in = torch.zeros(V + 2, dtype=torch.int32).pin_memory()
        self.pin_add = torch.zeros(V, dtype=torch.int32).pin_memory()
        self.pin_addv = torch.zeros(V, dtype=torch.float32).pin_memory()
        self.pin_cut = torch.zeros(V, dtype=torch.float32).pin_memory()
        self.pin_nadd = torch.zeros(1, dtype=torch.int32).pin_memory()

    def _alloc(self, R):
        self.cap = R
        self.zlat = torch.zeros(R, 64, device=self.dev, dtype=torch.float32)
        self.h3 = torch.zeros(R, self.d, device=self.dev, dtype=torch.float32)
        self.probs_dev = torch.zeros(R, self.V, device=self.dev, dtype=torch.float32)

    # ------------------------------------------------------------------ batched encoder / decoder
    def encode_lists(self, lists):
        """model.encoder(x) for R cubes given as card-index lists -> [R, 64] fp32 (device)."""
        R = len(lists)
        lists = [np.unique(np.asarray(l, np.int64)).astype(np.int32) for l in lists]
        row_ptr = np.zeros(R + 1, np.int32)
        row_ptr[1:] = np.cumsum([len(l) for l in lists])
        idx = np.concatenate(lists) if R else np.zeros(0, np.int32)
        with torch.cuda.stream(self.stream):
            rp = torch.from_numpy(row_ptr).to(self.dev, non_blocking=True)
            ix = torch.from_numpy(idx if len(idx) else np.zeros(1, np.int32)).to(self.dev, non_blocking=True)
            z = torch.zeros(R, 64, device=self.dev, dtype=torch.float32)
            L.call('cc_infer_encode_fp32', L.ptr(self.params), self.V, self.d, R, L.ptr(rp), L.ptr(ix),
                   L.ptr(z), L.stream_ptr(self.stream))
        self.stream.synchronize()
        return z

    def decode(self, z):
        """model.decoder(z): [R, 64] -> sigmoid probabilities [R, V] fp32 (device)."""
        z = torch.as_tensor(z, dtype=torch.float32).to(self.dev).contiguous()
        R = z.shape[0]
        with torch.cuda.stream(self.stream):
            h3 = torch.zeros(R, self.d, device=self.dev, dtype=torch.float32)
            out = torch.zeros(R, self.V, device=self.dev, dtype=torch.float32)
            L.call('cc_infer_decode_fp32', L.ptr(self.params), self.V, self.d, R, L.ptr(z), L.ptr(h3),
                   L.ptr(out), L.stream_ptr(self.stream))
        self.stream.synchronize()
        return out

    # ------------------------------------------------------------------ single-cube request
    def recommend(self, cube_indices, amount, want_probs=False, want_order=False):
        """ml_recommend.py:78-108 for one cube.  Returns dict with
        additions (card idx, descending), add_vals, cut_vals (per cube index, input order),
        and optionally the full probability vector / ranking."""
        ci = np.asarray(cube_indices, np.int64)
        uniq = np.unique(ci).astype(np.int32)
        n = len(uniq)
        amount = int(amount)
        want = min(max(amount, 1), self.V)
        with self.lock:
            s = L.stream_ptr(self.stream)
            with torch.cuda.stream(self.stream):
                self.pin_in[0] = 0
                self.pin_in[1] = n
                self.pin_in[2:2 + n] = torch.from_numpy(uniq)
                self.idx_dev[:2 + n].copy_(self.pin_in[:2 + n], non_blocking=True)
                L.call('cc_infer_encode_fp32', L.ptr(self.params), self.V, self.d, 1, L.ptr(self.idx_dev),
                       L.ptr(self.idx_dev[2:]), L.ptr(self.zlat), s)
                L.call('cc_infer_decode_fp32', L.ptr(self.params), self.V, self.d, 1, L.ptr(self.zlat),
                       L.ptr(self.h3), L.ptr(self.probs_dev), s)
                L.call('cc_topn', L.ptr(self.probs_dev), self.V, L.ptr(self.idx_dev[2:]), n, amount,
                       L.ptr(self.additions), L.ptr(self.n_add), L.ptr(self.add_vals), L.ptr(self.cut_vals),
                       L.ptr(self.order) if want_order else None, L.ptr(self.topn_ws), s)
                self.pin_nadd.copy_(self.n_add, non_blocking=True)
                self.pin_add[:want].copy_(self.additions[:want], non_blocking=True)
                self.pin_addv[:want].copy_(self.add_vals[:want], non_blocking=True)
                if n:
                    self.pin_cut[:n].copy_(self.cut_vals[:n], non_blocking=True)
                probs = self.probs_dev[0].clone() if want_probs else None
                order = self.order.clone() if want_order else None
            self.stream.synchronize()
            k = int(self.pin_nadd[0])
            cut_by_card = dict(zip(uniq.tolist(), self.pin_cut[:n].tolist()))
            out = {
                'additions': self.pin_add[:k].numpy().copy(),
                'add_vals': self.pin_addv[:k].numpy().copy(),
                'cut_vals': np.array([cut_by_card[int(c)] for c in ci], np.float32),
            }
        if want_probs:
            out['probs'] = probs.cpu().numpy()
        if want_order:
            out['order'] = order.cpu().numpy()
        return out
