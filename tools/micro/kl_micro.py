#!/usr/bin/env python3
"""Micro-benchmark of the fused D2 path (cc_dec_softmax_kl_dw: stats, merge, main, fix kernels) at
the bench's +KL shape (|V| = 22,000, d = 256, 512 regulariser rows, bf16): HIP events around N
back-to-back launches of the D2 call on the Trainer's own buffers.  Run under rocprofv3 for the
per-kernel split.   python tools/micro/kl_micro.py [--rows N] [--iters K]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--mode', default='sampled')
    a = ap.parse_args()
    from cubecobrarecommender_amd import _lib as L
    from cubecobrarecommender_amd.adjacency import adjacency_normalised_gpu
    from cubecobrarecommender_amd.layout import glorot_flat
    from cubecobrarecommender_amd.synthetic import neg_sampler_from_csr, synthetic_cubes
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    V, d, B = 22000, 256, 512
    ip, ix = synthetic_cubes(8192, V, device='cuda')
    ns = neg_sampler_from_csr(ip, ix, V)
    Mt = adjacency_normalised_gpu(ip, ix, V)
    tr = Trainer(TrainConfig(V=V, d=d, batch_size=B, reg=0.1, dtype='bf16', reg_mode=a.mode),
                 DeviceDataset(csr=(ip, ix), num_cards=V, neg_sampler=ns, y_mtx=Mt), params_flat=glorot_flat(V, d, 1))
    tr.set_epoch_permutation(np.random.default_rng(0).permutation(8192))
    assert tr.fused_reg
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    calls = []
    orig = L.call

    def spy(name, *args):
        if name == 'cc_dec_softmax_kl_dw':
            calls.append(args)
        return orig(name, *args)
    L.call = spy
    tr.forward_backward()
    L.call = orig
    torch.cuda.synchronize()
    args = calls[0]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        L.call('cc_dec_softmax_kl_dw', *args)
    e1.record()
    torch.cuda.synchronize()
    print(f'cc_dec_softmax_kl_dw rows={tr.Breg}: {e0.elapsed_time(e1) / a.iters * 1e3:.1f} us per call')


if __name__ == '__main__':
    main()
