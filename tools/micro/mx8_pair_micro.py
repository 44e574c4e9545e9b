"""Config 5's BCE-product launch (cc_gemm_mx8_bce_q2: the BCE product's 172 tiles + the regulariser
logits' 172 tiles in one 344-block launch on 256 CUs) against its halves and against the
regulariser logits split over K (dev tool): HIP-event averages per variant at d = 1024,
|V| = 22,000, B = 512, interleaved, each after a 512 MB read that evicts the caches."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402
from tools.micro.mx8_bench import (B, V, d, Vp, D3q, D3qs, WoT8, WoT8s, dZq, dZqs, dZtq, dZtqs, bias, gbias,  # noqa: E402
                                   ybits, part, Z2, args)


def main():
    split = torch.empty(4 * B * V, device='cuda')

    def bce():
        return args(B, V, d, D3q, d, WoT8, d, L.CC_EPI_BCE, sa=D3qs, sb=WoT8s, bias=bias, y_bits=ybits,
                    loss_partials=part)

    def bce_q2(g2):
        L.call('cc_gemm_mx8_bce_q2', C.byref(bce()), L.ptr(dZq), Vp, L.ptr(dZqs), L.ptr(dZtq), B, L.ptr(dZtqs),
               L.ptr(gbias), C.byref(g2) if g2 is not None else None, L.stream_ptr())

    reg = args(B, V, d, D3q, d, WoT8, d, L.CC_EPI_STORE, sa=D3qs, sb=WoT8s, bias=bias, Cf=Z2)
    reg_s2 = args(B, V, d, D3q, d, WoT8, d, L.CC_EPI_SPLITK, sa=D3qs, sb=WoT8s, Cf=split, splits=2)
    reg_s4 = args(B, V, d, D3q, d, WoT8, d, L.CC_EPI_SPLITK, sa=D3qs, sb=WoT8s, Cf=split, splits=4)
    variants = {
        'bce_q alone (172)': lambda: bce_q2(None),
        'reg logits alone (172)': lambda: L.call('cc_gemm', C.byref(reg), L.stream_ptr()),
        'reg logits split2 (344)': lambda: L.call('cc_gemm', C.byref(reg_s2), L.stream_ptr()),
        'pair bce + reg (344)': lambda: bce_q2(reg),
        'pair bce + reg split2 (516)': lambda: bce_q2(reg_s2),
        'pair bce + reg split4 (860)': lambda: bce_q2(reg_s4),
    }
    big = torch.empty(128 << 20, device='cuda')
    times = {k: [] for k in variants}
    for rep in range(25):
        for k, f in variants.items():
            big.mul_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            times[k].append((e0, e1))
    torch.cuda.synchronize()
    for k, ev in times.items():
        us = [a.elapsed_time(b) * 1e3 for a, b in ev[5:]]
        print(f'{k:30s} {np.mean(us):7.2f} us (min {np.min(us):.2f})', flush=True)


if __name__ == '__main__':
    main()
