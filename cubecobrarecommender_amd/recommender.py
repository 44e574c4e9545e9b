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

GRAPH_MAX_IDS = 4096   # cube ids per request the captured graph's H2D carries


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
        self.probs_dev = torch.zeros(V, device=self.dev, dtype=torch.float32)
        self.ws = torch.zeros(int(L.lib().cc_recommend_ws_size(V, d)) // 4 + 64,
                              device=self.dev, dtype=torch.int32)
        # request I/O: req = {n, amount, ids[n]}, res = {n_add, additions, add_vals, cut_vals}
        self.cap = min(V, GRAPH_MAX_IDS)
        self.req_dev = torch.zeros(2 + V, device=self.dev, dtype=torch.int32)
        self.res_dev = torch.zeros(1 + 2 * V + V, device=self.dev, dtype=torch.int32)
        self.pin_req = torch.zeros(2 + V, dtype=torch.int32).pin_memory()
        self.pin_res = torch.zeros(1 + 2 * V + V, dtype=torch.int32).pin_memory()
        self._req_np = self.pin_req.numpy()
        self._res_np = self.pin_res.numpy()
        self._graph = None
        # the request graph runs on the library's own non-blocking stream: every allocation and
        # fill above (issued on torch's stream) must be complete before it can run
        torch.cuda.synchronize(self.dev)

    def __del__(self):
        g = getattr(self, '_graph', None)
        if g is not None:
            try:
                L.lib().cc_recommend_graph_destroy(g)
            except Exception:
                pass

    def _graph_handle(self):
        if self._graph is None:
            h = L.C.c_void_p()
            L.call('cc_recommend_graph_create', L.ptr(self.params), self.V, self.d, L.ptr(self.pin_req),
                   L.ptr(self.req_dev), self.cap, L.ptr(self.ws), L.ptr(self.probs_dev), L.ptr(self.res_dev),
                   L.C.byref(h))
            self._graph = h
        return self._graph

    # ------------------------------------------------------------------ batched encoder / decoder
    def encode_lists(self, lists):
        """model.encoder(x) for R cubes given as card-index lists -> [R, 64] fp32 (device)."""
        R = len(lists)
        lists = [np.unique(np.asarray(l, np.int64)).astype(np.int32) for l in lists]
        row_ptr = np.zeros(R + 1, np.int32)
        row_ptr[1:] = np.cumsum([len(l) for l in lists])
        max_n = max([len(l) for l in lists], default=0)
        idx = np.concatenate(lists) if R else np.zeros(0, np.int32)
        with torch.cuda.stream(self.stream):
            rp = torch.from_numpy(row_ptr).to(self.dev, non_blocking=True)
            ix = torch.from_numpy(idx if len(idx) else np.zeros(1, np.int32)).to(self.dev, non_blocking=True)
            z = torch.zeros(R, 64, device=self.dev, dtype=torch.float32)
            ws = torch.empty(int(L.lib().cc_infer_encode_ws_size(R, self.d, max_n)) // 4 + 4,
                             device=self.dev, dtype=torch.float32)
            L.call('cc_infer_encode_fp32', L.ptr(self.params), self.V, self.d, R, L.ptr(rp), L.ptr(ix),
                   max_n, L.ptr(ws), L.ptr(z), L.stream_ptr(self.stream))
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
        """ml_recommend.py:78-108 for one cube.  Returns dict with additions (card idx,
        descending), add_vals, cut_vals (per cube index, input order), and optionally the full
        probability vector / ranking.  Cubes of up to GRAPH_MAX_IDS distinct cards replay the
        captured request graph (one launch, one D2H); larger ones run the same kernels directly."""
        ci = np.asarray(cube_indices, np.int64)
        uniq = np.unique(ci).astype(np.int32)
        n = len(uniq)
        amount = int(amount)
        want = min(max(amount, 1), self.V - n)
        words = 1 + 2 * want + n
        with self.lock:
            req = self._req_np
            req[0] = n
            req[1] = amount
            req[2:2 + n] = uniq
            if n <= self.cap:
                L.call('cc_recommend_graph_run', self._graph_handle(), L.ptr(self.pin_res), words)
            else:
                with torch.cuda.stream(self.stream):
                    self.req_dev[:2 + n].copy_(self.pin_req[:2 + n], non_blocking=True)
                    L.call('cc_recommend_fp32', L.ptr(self.params), self.V, self.d, L.ptr(self.req_dev), n,
                           L.ptr(self.ws), L.ptr(self.probs_dev), L.ptr(self.res_dev), L.stream_ptr(self.stream))
                    self.pin_res[:words].copy_(self.res_dev[:words], non_blocking=True)
                self.stream.synchronize()
            r = self._res_np
            k = int(r[0])
            cut = r[1 + 2 * want:1 + 2 * want + n].view(np.float32)
            out = {
                'additions': r[1:1 + k].copy(),
                'add_vals': r[1 + want:1 + want + k].view(np.float32).copy(),
                'cut_vals': cut[np.searchsorted(uniq, ci)].copy() if n else np.zeros(0, np.float32),
            }
            probs = order = None
            if want_probs or want_order:
                probs = self.probs_dev.clone()   # the graph ran on its own stream and was waited for
            if want_order:
                order = self._full_order(probs, uniq, amount)
        if want_probs:
            out['probs'] = probs.cpu().numpy()
        if want_order:
            out['order'] = order
        return out

    def _full_order(self, probs, uniq, amount):
        """The complete ranking (cc_topn with `order`; tests and tools only)."""
        V, dev = self.V, self.dev
        n = len(uniq)
        want = min(max(amount, 1), V)
        ci = torch.from_numpy(uniq if n else np.zeros(1, np.int32)).to(dev)
        adds = torch.zeros(want, device=dev, dtype=torch.int32)
        addv = torch.zeros(want, device=dev)
        cutv = torch.zeros(max(n, 1), device=dev)
        nadd = torch.zeros(1, device=dev, dtype=torch.int32)
        order = torch.zeros(V, device=dev, dtype=torch.int32)
        ws = torch.zeros(int(L.lib().cc_topn_workspace_size(V)) // 4 + 64, device=dev, dtype=torch.int32)
        L.call('cc_topn', L.ptr(probs), V, L.ptr(ci), n, amount, L.ptr(adds), L.ptr(nadd), L.ptr(addv),
               L.ptr(cutv), L.ptr(order), L.ptr(ws), L.stream_ptr())
        torch.cuda.synchronize()
        return order.cpu().numpy()
