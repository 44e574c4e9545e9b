"""Time cc_embed_gather_fwd on a bench-shaped batch (synthetic Zipf cubes, V=22000, d=256, R=512)
for the kernel variants selected by CCREC_GATHER2 (dev tool).  Prints us per launch and the max
abs difference against the first variant's output."""
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def run_variant():
    from cubecobrarecommender_amd import _lib as L
    from cubecobrarecommender_amd.synthetic import synthetic_cubes
    V, d, R = 22000, 256, 512
    indptr, indices = synthetic_cubes(R, V, seed=5, device='cuda')
    ip, ix = np.asarray(indptr), np.asarray(indices)
    x_cap = 1300
    cnt = np.diff(ip).astype(np.int32)
    xi = np.zeros((R, x_cap), np.int32)
    for r in range(R):
        xi[r, :cnt[r]] = ix[ip[r]:ip[r + 1]]
    x_cnt, x_idx = torch.from_numpy(cnt).cuda(), torch.from_numpy(xi).cuda()
    g = torch.Generator(device='cuda').manual_seed(0)
    table = (torch.randn(V, d, device='cuda', generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(d, device='cuda', generator=g) * 0.1
    out = torch.zeros(R, d, device='cuda', dtype=torch.bfloat16)
    big = torch.empty(64 << 20, device='cuda', dtype=torch.int32)   # evicts L2 / MALL between launches
    fn = lambda: L.call('cc_embed_gather_fwd', L.CC_BF16, L.ptr(table), L.ptr(bias), V, d, R, L.ptr(x_cnt),
                        L.ptr(x_idx), x_cap, L.ptr(out), L.stream_ptr())
    ts = []
    for it in range(40):
        big.add_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(a.elapsed_time(b) * 1e3)
    ref = (table.float()[torch.from_numpy(ix.astype(np.int64)).cuda()])
    seg = torch.repeat_interleave(torch.arange(R, device='cuda'), torch.from_numpy(cnt.astype(np.int64)).cuda())
    want = torch.relu(torch.zeros(R, d, device='cuda').index_add_(0, seg, ref) + bias)
    err = (out.float() - want).abs().max().item()
    print(f"gather2={os.environ.get('CCREC_GATHER2')} {np.median(ts):.1f} us (cold L2/MALL), max err {err:.3g}",
          flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1:
        run_variant()
    else:
        for v in ('0', '44', '48', '84', '88', '46', '86'):
            subprocess.run([sys.executable, __file__, 'x'], env=dict(os.environ, CCREC_GATHER2=v), check=True)
