"""CPU tests (gloo, world_size 2) of the data-parallel host logic."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from cubecobrarecommender_amd import distributed as D
    w, r, dev = D.init(backend='gloo')
    assert (w, r) == (world, rank)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    D.allreduce_grads(g, n=8)
    perm = np.random.default_rng(0).permutation(64)
    cubes = [D.rank_cubes(perm, bi, 4, rank, world).tolist() for bi in range(8)]
    q.put((rank, g.tolist(), cubes))
    D.finish()


def test_gloo_world2_allreduce_and_sharding():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (g, c)) for r, g, c in [q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    want = [i * 1.5 for i in range(8)] + [8.0, 9.0]        # mean of x*1 and x*2 on the first 8
    assert res[0][0] == pytest.approx(want[:8] + [8.0, 9.0])
    assert res[1][0][:8] == pytest.approx(want[:8])
    # ranks take disjoint slices; together they cover the global batch in order
    perm = np.random.default_rng(0).permutation(64)
    for bi in range(8):
        both = res[0][1][bi] + res[1][1][bi]
        assert both == perm[bi * 8:(bi + 1) * 8].tolist()
