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


def _adam(p, m, v, g, t, lr=1e-3, b1=0.9, b2=0.999, eps=1e-7):
    """TF ResourceApplyAdam in float32 torch ops, in place."""
    m.add_((g - m) * (1 - b1))
    v.add_((g * g - v) * (1 - b2))
    lr_t = lr * (1 - b2 ** t) ** 0.5 / (1 - b1 ** t)
    p.sub_(lr_t * m / (v.sqrt() + eps))


class _FakeTrainer:
    def __init__(self, world, rank, with_reg, shadow=False, chunks=1):
        from types import SimpleNamespace
        from cubecobrarecommender_amd.layout import Layout
        self.cfg = SimpleNamespace(world=world, rank=rank)
        self.layout = Layout(300, 64, align=world * 64, group_biases=shadow, w1_chunks=chunks)
        self.use_reg = with_reg
        n = self.layout.total
        gen = torch.Generator().manual_seed(7)
        self.params = torch.randn(n, generator=gen)
        self.m = torch.zeros(n)
        self.v = torch.zeros(n)
        self.grads = torch.randn(n, generator=torch.Generator().manual_seed(100 + rank))
        self.shadow = self.params.to(torch.bfloat16) if shadow else None


def _zero_worker(rank, world, port, q, shadow=False, chunks=1):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from cubecobrarecommender_amd import distributed as D
    from cubecobrarecommender_amd.zero import ShardedStep
    D.init(backend='gloo')
    tr = _FakeTrainer(world, rank, with_reg=True, shadow=shadow, chunks=chunks)
    zs = ShardedStep(tr)
    assert zs.shadow_gather == shadow
    for t in (1, 2):
        def adam_fn(lo, n, g, t=t):
            _adam(tr.params[lo:lo + n], tr.m[lo:lo + n], tr.v[lo:lo + n], g, t)
            if tr.shadow is not None:     # cc_adam_dense writes the bf16 shadow of its range
                tr.shadow[lo:lo + n] = tr.params[lo:lo + n].to(torch.bfloat16)
        zs.step(lambda: None, lambda: None, lambda: None, adam_fn, lambda lo, hi: None)
    sh = tr.shadow.float().numpy().copy() if shadow else None
    bias = tr.params[tr.layout.bias_lo:].numpy().copy() if shadow else None
    zs.gather_state()
    q.put((rank, tr.params.numpy().copy(), tr.m.numpy().copy(), tr.v.numpy().copy(), sh, bias))
    D.finish()


@pytest.mark.parametrize('shadow,chunks', [(False, 1), (True, 1), (True, 3)])
def test_gloo_world2_sharded_adam_equals_allreduce_adam(shadow, chunks):
    """ZeRO-1 step (bucketed reduce-scatter, Adam on the rank's shard, all-gather; zero.py)
    leaves every rank with exactly the parameters of a full Adam on the averaged gradient.
    shadow: the bf16 path's grouped-bias layout — the kernels' bf16 shadow is all-gathered and the
    biases bucket all-reduced (Adam on every rank): after the steps every rank holds the exact
    shadow and fp32 biases, and gather_state() completes the fp32 kernels, m and v.  chunks: W1's
    gradient exchanged in row-chunk buckets (the bf16 layout's early output-layer bucket too)."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 7 + 11 * shadow + 23 * chunks) % 1000
    ps = [ctx.Process(target=_zero_worker, args=(r, world, port, q, shadow, chunks)) for r in range(world)]
    for p in ps:
        p.start()
    res = {r: rest for r, *rest in [q.get(timeout=120) for _ in ps]}
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    ref = _FakeTrainer(world, 0, with_reg=True, shadow=shadow, chunks=chunks)
    g = sum(_FakeTrainer(world, r, True, shadow=shadow, chunks=chunks).grads for r in range(world)) * (1.0 / world)
    for t in (1, 2):
        _adam(ref.params, ref.m, ref.v, g, t)
    for r in range(world):
        pp, mm, vv, sh, bias = res[r]
        np.testing.assert_array_equal(pp, ref.params.numpy())
        np.testing.assert_array_equal(mm, ref.m.numpy())
        np.testing.assert_array_equal(vv, ref.v.numpy())
        if shadow:
            np.testing.assert_array_equal(sh, ref.params.to(torch.bfloat16).float().numpy())
            np.testing.assert_array_equal(bias, ref.params[ref.layout.bias_lo:].numpy())


@pytest.mark.parametrize('V,d,world,chunks', [(22000, 256, 8, 4), (22000, 1024, 8, 4), (300, 64, 2, 3),
                                              (2500, 256, 1, 4), (3000, 1024, 2, 4), (301, 64, 4, 2)])
def test_grouped_layout_buckets(V, d, world, chunks):
    """The data-parallel bf16 / fp8 layout (layout.Layout(group_biases=True)): the buckets are
    disjoint, aligned to world*64, in backward order (output layers, W1 chunks, biases),
    cover every tensor with the regulariser and skip exactly the decoder_for_reg tensors without
    it; W1's row chunks tile [V, d] contiguously (the towers in the last chunk's bucket); packing
    round-trips every tensor."""
    from cubecobrarecommender_amd.layout import NAMES, Layout
    lay = Layout(V, d, align=world * 64, group_biases=True, w1_chunks=chunks)
    a = world * 64
    for with_reg in (True, False):
        bk = lay.buckets(with_reg)
        names = [n for n, _, _ in bk]
        assert names[0] == 'output_layers' and names[-1] == 'biases'
        assert names[1:-1] == [f'w1_{i}' for i in range(len(lay.w1_chunks))]
        spans = sorted((lo, hi) for _, lo, hi in bk)
        assert all(lo % a == 0 and hi % a == 0 and lo < hi for lo, hi in spans)
        assert all(h0 <= l1 for (_, h0), (l1, _) in zip(spans, spans[1:]))
        for n in NAMES:
            o, shape = lay.entries[n]
            size = int(np.prod(shape))
            inside = [b for b, lo, hi in bk if lo <= o and o + size <= hi]
            skip = not with_reg and n.startswith('decoder_for_reg/') and n.endswith('/kernel')
            if n == 'encoder/encoded_1/kernel':   # W1: the chunk buckets (the last also holds the towers)
                w1b = [(lo, hi) for b, lo, hi in bk if b.startswith('w1_')]
                assert w1b[0][0] == o and o + size <= w1b[-1][1]
                assert [lo for lo, _ in w1b] == [r0 * d for r0, _ in lay.w1_chunks]
                continue
            assert len(inside) == (0 if skip else 1), (n, with_reg, inside)
    assert lay.w1_chunks[0][0] == 0 and lay.w1_chunks[-1][1] == V
    assert all(r1 == r0n for (_, r1), (r0n, _) in zip(lay.w1_chunks, lay.w1_chunks[1:]))
    rng = np.random.default_rng(0)
    P = {n: rng.standard_normal(lay.shape(n)).astype(np.float32) for n in NAMES}
    back = lay.unpack(lay.pack(P))
    assert all(np.array_equal(back[n], P[n]) for n in NAMES)
