"""Where does the Adam + F launch's time go?  Eager HIP-event timings at the bench's BCE shape
(V = 22,000, d = 256, B = 512) of: the launch as the step issues it (Adam over the rest ranges +
packed tower images + next-step F), F alone, the same Adam element count without F / packs
(cc_adam_dense on scratch), with F but no packs (cc_adam_noise on scratch), and Adam alone at a
few sizes (the achieved HBM rate curve).

    python tools/micro/adam_place_micro.py"""
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


def main():
    from cubecobrarecommender_amd.layout import glorot_flat
    from cubecobrarecommender_amd.synthetic import neg_sampler_from_csr, synthetic_cubes
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    V, d, B, C = 22000, 256, 512, 65536
    indptr_t, indices_t = synthetic_cubes(C, V, seed=7, device='cuda')
    indptr, indices = np.asarray(indptr_t), np.asarray(indices_t)
    data = DeviceDataset(csr=(indptr, indices), num_cards=V, neg_sampler=neg_sampler_from_csr(indptr, indices, V),
                         device='cuda')
    tr = Trainer(TrainConfig(V=V, d=d, batch_size=B, reg=0.0, dtype='bf16', seed=5, fuse_w1_adam=True,
                             wo_adam_in_tower=True), data,
                 params_flat=glorot_flat(V, d, seed=3))
    tr.set_epoch_permutations(np.random.default_rng(1).permutation(C).astype(np.int32)[None, :])
    for _ in range(3):
        tr.forward_backward()
        tr.apply()
    torch.cuda.synchronize()
    o = tr.w1_off
    (a0, b0), (a1, b1) = tr.rest_ranges[0], (tr.rest_ranges + [(o, o)])[1]
    n = (b0 - a0) + (b1 - a1)
    print(f'rest ranges {tr.rest_ranges} (w1_off {o}): {n} elements, {n * 30 / 1e6:.1f} MB algorithmic')
    na = tr._noise_args()
    res = {}
    res['adam+F+pack (step)'] = timeit(lambda: tr.apply_adam())
    res['F alone'] = timeit(lambda: L.call('cc_noise_next', L.C.byref(na), tr.batches_per_epoch, L.stream_ptr(None)))
    for nn in (n, 2 * n, 4 * n, 11_520_000):
        p, m, v, g = (torch.rand(nn, device='cuda') for _ in range(4))
        sh = torch.zeros(nn, dtype=torch.int16, device='cuda')
        args = (L.ptr(p), L.ptr(m), L.ptr(v), L.ptr(g), L.ptr(sh), nn)
        us = timeit(lambda: L.call('cc_adam_dense', *args, L.ptr(tr.state), 1e-3, 0.9, 0.999, 1e-7, L.stream_ptr(None)))
        res[f'adam alone n={nn}'] = f'{us:.1f} us = {nn * 30 / us / 1e6:.2f} TB/s'
        if nn == n:
            res['adam+F no pack'] = timeit(lambda: L.call('cc_adam_noise', *args, 1e-3, 0.9, 0.999, 1e-7, L.C.byref(na),
                                                          tr.batches_per_epoch, L.stream_ptr(None)))
        del p, m, v, g, sh
    for k, v in res.items():
        print(f'{k:28s} {v if isinstance(v, str) else f"{v:.1f} us"}')


if __name__ == '__main__':
    main()
