"""Time the GPU co-occurrence graph (cc_adjacency) on a synthetic corpus.

python tools/adjacency_bench.py [--V 22000] [--C 65536] [--reps 5] [--outputs Mt]
Prints one JSON line: ms per build (events around cc_adjacency: Xt scatter + card stats +
symmetric FP4 GEMM + fused normalisation), the FP4 MFMA rate of the GEMM kernel counted as
the upper-triangle tiles it actually multiplies, and the dense-equivalent rate 2*V^2*K.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def corpus(V, C, seed=0):
    rng = np.random.default_rng(seed)
    pop = 1.0 / (1.0 + rng.permutation(V)) ** 0.8
    cdf = np.cumsum(pop / pop.sum())
    sizes = rng.integers(180, 721, size=C)
    # with-replacement Zipf draws (duplicates collapse in the kernel, as in the dense matrix)
    idx = np.searchsorted(cdf, rng.random(int(sizes.sum()))).clip(0, V - 1).astype(np.int32)
    indptr = np.zeros(C + 1, np.int64)
    indptr[1:] = np.cumsum(sizes)
    return indptr, idx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--V', type=int, default=22000)
    ap.add_argument('--C', type=int, default=65536)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--chunk', type=int, default=0)
    ap.add_argument('--outputs', default='Mt')
    a = ap.parse_args()
    from cubecobrarecommender_amd.adjacency import adjacency_device, upload_lists
    t0 = time.time()
    indptr, idx = corpus(a.V, a.C)
    gen_s = time.time() - t0
    outs = tuple(a.outputs.split(','))
    rp, ix, C = upload_lists(indptr, idx, a.V)   # host validation + H2D, outside the timing
    adjacency_device(rp, ix, C, a.V, outs, chunk_cubes=a.chunk)  # warm-up (allocations, code)
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = adjacency_device(rp, ix, C, a.V, outs, chunk_cubes=a.chunk)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
        del r
    K = (a.C + 255) // 256 * 256
    nb = (a.V + 255) // 256
    tri_ops = 2.0 * 256 * 256 * K * nb * (nb + 1) / 2
    med = float(np.median(ms))
    print(json.dumps({'kernel': 'cc_adjacency', 'V': a.V, 'C': a.C, 'outputs': outs,
                      'ms_median': med, 'ms_all': ms,
                      'fp4_tops_issued': tri_ops / (med * 1e-3) / 1e12,
                      'dense_equiv_tops': 2.0 * a.V * a.V * a.C / (med * 1e-3) / 1e12,
                      'host_corpus_s': gen_s}))


if __name__ == '__main__':
    main()
