"""W1 gradient + Adam in isolation (dev tool): the cube rows only (R = 512), the reg rows by index
(cc_embed_grad_cs_adam_reg, nreg = 512 cards drawn from the bench's neg_sampler) and the reg rows as
bits (R = 1024), at V = 22,000, d = 256, with and without the bias row; HIP-event averages per
variant, interleaved; --warm: no cache eviction between launches."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402


def main():
    V, B = 22000, 512
    d = int(sys.argv[sys.argv.index('--d') + 1]) if '--d' in sys.argv else 256
    pk = int(sys.argv[sys.argv.index('--packed') + 1]) if '--packed' in sys.argv else 1
    from cubecobrarecommender_amd.synthetic import synthetic_cubes, neg_sampler_from_csr
    ip, ix = synthetic_cubes(65536, V, seed=20250301, device='cpu')
    ns = np.asarray(neg_sampler_from_csr(ip, ix, V), np.float64)
    rng = np.random.default_rng(1)
    reg = rng.choice(V, B, p=ns / ns.sum()).astype(np.int32)
    R2 = 2 * B
    RP = R2
    X = rng.random((B, V)) < 0.02
    xt2 = np.zeros((V, R2 // 32), np.uint32)
    rr, cc = np.nonzero(X)
    np.bitwise_or.at(xt2, (cc, rr // 32), (np.uint32(1) << (rr % 32).astype(np.uint32)))
    rr2 = B + np.arange(B)
    np.bitwise_or.at(xt2, (reg, rr2 // 32), (np.uint32(1) << (rr2 % 32).astype(np.uint32)))
    xt1 = np.ascontiguousarray(xt2[:, :B // 32])
    xb1 = torch.from_numpy(xt1.view(np.int32)).cuda()
    xb2 = torch.from_numpy(xt2.view(np.int32)).cuda()
    g = (torch.randn(RP, d, device='cuda') * 0.1).to(torch.bfloat16)
    gP = (g.view(RP // 16, 2, 8, d // 32, 32).permute(3, 0, 1, 4, 2).contiguous() if pk else
          g.t().contiguous())   # packed fragment image, or dPre1^T [d][RP]
    rid = torch.from_numpy(reg).cuda()
    p = torch.randn(V * d, device='cuda') * 0.02
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    sh = p.to(torch.bfloat16)
    bg = torch.zeros(d, device='cuda')
    st = torch.zeros(4, dtype=torch.int64, device='cuda')
    s = L.stream_ptr()
    def reg_call(bias):
        return lambda: L.call('cc_embed_grad_cs_adam_reg', L.ptr(gP), pk, V, d, B, RP, L.ptr(xb1),
                              L.ptr(bg) if bias else None, None, L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(sh),
                              L.ptr(st), 1e-3, 0.9, 0.999, 1e-7, L.ptr(rid), B, B // 16, s)

    def cube_call(bias):
        return lambda: L.call('cc_embed_grad_cs_adam', L.ptr(gP), pk, V, d, B, RP, L.ptr(xb1),
                              L.ptr(bg) if bias else None, None, L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(sh),
                              L.ptr(st), 1e-3, 0.9, 0.999, 1e-7, s)
    variants = {
        'cubes_only_nobias': cube_call(False),
        'reg_by_index_nobias': reg_call(False),
        'cubes_only_R512': lambda: L.call('cc_embed_grad_cs_adam', L.ptr(gP), pk, V, d, B, RP, L.ptr(xb1), L.ptr(bg),
                                          None, L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(sh), L.ptr(st), 1e-3, 0.9,
                                          0.999, 1e-7, s),
        'reg_by_index': lambda: L.call('cc_embed_grad_cs_adam_reg', L.ptr(gP), pk, V, d, B, RP, L.ptr(xb1), L.ptr(bg),
                                       None, L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(sh), L.ptr(st), 1e-3, 0.9, 0.999,
                                       1e-7, L.ptr(rid), B, B // 16, s),
        'reg_as_bits_R1024': lambda: L.call('cc_embed_grad_cs_adam', L.ptr(gP), pk, V, d, R2, RP, L.ptr(xb2),
                                            L.ptr(bg), None, L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(sh), L.ptr(st),
                                            1e-3, 0.9, 0.999, 1e-7, s),
    }
    times = {k: [] for k in variants}
    big = torch.empty(256 << 20, device='cuda')   # evicts the MALL between launches, as a step does
    warm = '--warm' in sys.argv                    # (or not: p / m / v stay in the MALL)
    for rep in range(40):
        for k, f in variants.items():
            if not warm:
                big.mul_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            times[k].append((e0, e1))
    torch.cuda.synchronize()
    for k, ev in times.items():
        us = [a.elapsed_time(b) * 1e3 for a, b in ev[5:]]
        print(f'{k:20s} {np.mean(us):7.2f} us (min {np.min(us):.2f})', flush=True)


if __name__ == '__main__':
    main()
