"""Time the fused tower kernels alone at d=256 bf16 for several row counts R (dev tool):
is the chain latency-bound (time flat in R) or throughput-bound?"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402


def setup(d, R, packed):
    B = R
    tdt = torch.bfloat16
    dims = [(d, 256), (256, 128), (128, 64), (64, 128), (128, 256), (256, d)]
    W = [torch.randn(*dims[l if l < 6 else l - 3], device='cuda').mul(0.05).to(tdt) for l in range(9)]
    Wt = [torch.zeros(w.shape[1], w.shape[0], device='cuda', dtype=tdt) for w in W]
    bias = [torch.randn(w.shape[1], device='cuda') * 0.1 for w in W]
    widths = [d, 256, 128, 64, 128, 256, d]
    act = [torch.randn(R, d, device='cuda').to(tdt)] + [torch.zeros(R, w, device='cuda', dtype=tdt) for w in widths[1:]]
    act6t = torch.zeros(d, R, device='cuda', dtype=tdt)
    gD3 = torch.randn(R, d, device='cuda').to(tdt)
    gact = [torch.zeros(R, w, device='cuda', dtype=tdt) for w in (256, 128, 64, 128, 256)]
    gpre1 = torch.zeros(R, d, device='cuda')
    gpre1t = torch.zeros(d, (R + 63) // 64 * 64, device='cuda', dtype=tdt)
    slab = torch.zeros((R // 32) * int(L.lib().cc_tower_slab_elems(d)), device='cuda')
    gw = [torch.zeros(w.shape, device='cuda') for w in W]
    gb = [torch.zeros(w.shape[1], device='cuda') for w in W]
    t = L.TowerArgs(dtype=L.CC_BF16, d=d, B=B, R=R)
    for l in range(9):
        t.w[l], t.wt[l], t.b[l] = W[l].data_ptr(), Wt[l].data_ptr(), bias[l].data_ptr()
        t.gw[l], t.gb[l] = gw[l].data_ptr(), gb[l].data_ptr()
    for a in range(7):
        t.act[a] = act[a].data_ptr()
    t.act6t = act6t.data_ptr()
    t.gD3, t.gpre1, t.slab = gD3.data_ptr(), gpre1.data_ptr(), slab.data_ptr()
    t.gpre1t = gpre1t.data_ptr()
    for a in range(5):
        t.gact[a] = gact[a].data_ptr()
    wp = [torch.zeros(2, w.numel(), device='cuda', dtype=tdt) for w in W]
    if packed:
        for l in range(9):
            t.wpf[l], t.wpb[l] = wp[l][0].data_ptr(), wp[l][1].data_ptr()
    keep = [W, Wt, bias, act, act6t, gD3, gact, gpre1, gpre1t, slab, gw, gb, wp]
    return t, keep


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


def main():
    d = int(os.environ.get('D', '256'))
    s = L.stream_ptr()
    for R, packed in ((32, 0), (32, 1), (512, 0), (512, 1), (1024, 1)):
        t, keep = setup(d, R, packed)
        L.call('cc_tower_transpose', ctypes.byref(t), s)
        res = {}
        for fn in ('cc_tower_fwd', 'cc_tower_bwd_chain', 'cc_tower_bwd_dw_direct'):
            res[fn] = timeit(lambda: L.call(fn, ctypes.byref(t), s))
        print(f'd={d} R={R} packed={packed}: ' + '  '.join(f'{k} {v:.1f} us' for k, v in res.items()), flush=True)


if __name__ == '__main__':
    main()
