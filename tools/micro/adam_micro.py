"""Time cc_adam_dense vs cc_adam_dense_t (no regions / Wo only / all regions) at the bench's
parameter count, and the E1 scatter kernels on a bench-shaped batch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cubecobrarecommender_amd import _lib as L  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


n = 11_520_000
V, d = 22000, 256
p, m, v, g = (torch.randn(n, device='cuda') for _ in range(4))
v.abs_()
sh = torch.zeros(n, dtype=torch.int16, device='cuda')
st = torch.zeros(4, dtype=torch.int64, device='cuda')
wo_off = 5_800_000 // 64 * 64
wot = torch.zeros(V, d, dtype=torch.int16, device='cuda')
tw = [torch.zeros(256, 256, dtype=torch.int16, device='cuda') for _ in range(6)]


def regions(kind):
    regs = []
    if kind == 'all':
        o = 100_032
        for t in tw:
            regs.append((o, 256, 256, t.data_ptr()))
            o += 65536 + 64
    if kind in ('wo', 'all'):
        regs.append((wo_off, d, V, wot.data_ptr()))
    arr = (L.AdamTRegion * max(1, len(regs)))()
    for i, (o, r, c, dst) in enumerate(regs):
        arr[i].off, arr[i].rows, arr[i].cols, arr[i].dst = o, r, c, dst
    return arr, len(regs)


res = {}
res['adam_dense'] = timeit(lambda: L.call('cc_adam_dense', L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(g), L.ptr(sh), n,
                                          L.ptr(st), 1e-3, 0.9, 0.999, 1e-7, L.stream_ptr()))
for kind in ('none', 'wo', 'all'):
    arr, k = regions(kind)
    res['adam_t_' + kind] = timeit(lambda: L.call('cc_adam_dense_t', L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(g),
                                                  L.ptr(sh), n, L.ptr(st), 1e-3, 0.9, 0.999, 1e-7, arr, k, 0,
                                                  L.stream_ptr()))
res['transpose_wo'] = timeit(lambda: L.call('cc_transpose', L.CC_BF16, L.ptr(sh[wo_off:]), d, V, L.ptr(wot),
                                            L.stream_ptr()))

# scatter: R = 512 rows, Zipf-ish bits
R = 512
rng = np.random.default_rng(0)
pop = 1.0 / (1.0 + rng.permutation(V)) ** 0.8
pop = np.minimum(1.0, pop / pop.sum() * 437)
bits = (rng.random((V, R)) < pop[:, None])
words = np.packbits(bits, axis=1, bitorder='little').view(np.uint32)
xt0 = torch.from_numpy(words.copy()).cuda()
xt = xt0.clone()
dpre = torch.randn(R, d, device='cuda')
grad = torch.zeros(V, d, device='cuda')
bg = torch.zeros(d, device='cuda')


def scat():
    xt.copy_(xt0)
    L.call('cc_embed_scatter_bwd', L.ptr(dpre), V, d, R, L.ptr(xt), L.ptr(grad), L.ptr(bg), L.stream_ptr())


res['xt_copy_only'] = timeit(lambda: xt.copy_(xt0))
res['scatter+copy'] = timeit(scat)
print({k: round(val, 2) for k, val in res.items()}, 'bits set', int(bits.sum()))
