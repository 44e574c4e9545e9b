"""Bit fingerprint of a few training steps under whichever library CCREC_LIB names (dev A/B:
a build variant that only re-times kernels must leave every bit unchanged).

    CCREC_LIB=.../libccrec_hip_x.so python tools/lib_bits.py OUT.json [--reg-mode full] [--V 22000]
Then compare two OUT files (python tools/lib_bits.py --cmp A.json B.json)."""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _h(t):
    import torch
    return hashlib.sha256(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out', nargs='?')
    ap.add_argument('--cmp', nargs=2)
    ap.add_argument('--V', type=int, default=22000)
    ap.add_argument('--d', type=int, default=256)
    ap.add_argument('--B', type=int, default=512)
    ap.add_argument('--reg', type=float, default=0.1)
    ap.add_argument('--reg-mode', default='full')
    ap.add_argument('--steps', type=int, default=2)
    a = ap.parse_args()
    if a.cmp:
        x, y = (json.load(open(f)) for f in a.cmp)
        diff = {k: (x[k], y.get(k)) for k in x if x[k] != y.get(k)}
        print('IDENTICAL' if not diff else f'DIFFER {diff}')
        sys.exit(0 if not diff else 1)
    import numpy as np
    import torch
    from cubecobrarecommender_amd.adjacency import adjacency_normalised_gpu
    from cubecobrarecommender_amd.layout import glorot_flat
    from cubecobrarecommender_amd.synthetic import neg_sampler_from_csr, synthetic_cubes
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    V, d, B, C = a.V, a.d, a.B, 4 * a.B
    indptr_t, indices_t = synthetic_cubes(C, V, seed=7, device='cuda')
    indptr, indices = np.asarray(indptr_t), np.asarray(indices_t)
    ns = neg_sampler_from_csr(indptr, indices, V)
    y_mtx = adjacency_normalised_gpu(indptr, indices, V, device='cuda') if a.reg > 0 else None
    data = DeviceDataset(csr=(indptr, indices), num_cards=V, neg_sampler=ns, y_mtx=y_mtx, device='cuda')
    cfg = TrainConfig(V=V, d=d, batch_size=B, reg=a.reg, dtype='bf16', seed=5, reg_mode=a.reg_mode)
    tr = Trainer(cfg, data, params_flat=glorot_flat(V, d, seed=3))
    tr.set_epoch_permutations(np.random.default_rng(1).permutation(C).astype(np.int32)[None, :])
    res = {}
    for s in range(a.steps):
        tr.forward_backward()
        torch.cuda.synchronize()
        res[f'grads{s}'] = _h(tr.grads)
        res[f'dZ{s}'] = _h(tr.dZout)
        res[f'loss{s}'] = repr(tr.losses())
        tr.apply()
    tr.flush()
    torch.cuda.synchronize()
    res['params'] = _h(tr.params)
    json.dump(res, open(a.out, 'w'), indent=1)
    print(os.environ.get('CCREC_LIB', 'default lib'), res)


if __name__ == '__main__':
    main()
