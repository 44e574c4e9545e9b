"""GPU test of the data-parallel training step end to end: two ranks (two processes on the one
GPU, gloo for the collectives) run Trainer.step() — bucketed reduce-scatter overlapped with the
towers' backward, Adam on each rank's shard, all-gathered parameters (zero.py) — eagerly and as
graph replays, and must match one process training on the concatenated batch."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.gpu_helpers import problem, rel_err

pytestmark = pytest.mark.gpu

V, D, B, C, W, STEPS = 700, 64, 32, 256, 2, 3


def _make(rank, world, batch, reg, P, lists, Mt, ns):
    from cubecobrarecommender_amd.layout import Layout
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    cfg = TrainConfig(V=V, d=D, batch_size=batch, reg=reg, dtype='fp32', seed=3, rank=rank, world=world)
    data = DeviceDataset(lists, V, y_mtx=Mt.astype(np.float32) if reg else None, neg_sampler=ns)
    tr = Trainer(cfg, data, params_flat=Layout(V, D).pack(P))
    tr.set_epoch_permutations(np.random.default_rng(4).permutation(C)[None, :])
    return tr


def _worker(rank, port, reg, graphs, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(W), LOCAL_RANK='0', HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        import torch.distributed as dist
        from oracle import model_ref
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=W)
        lists, Mt, ns = problem(3, C, V, (20, 40, 80))
        P = model_ref.init_params(V, D, seed=3, bias_std=0.01)
        tr = _make(rank, W, B, reg, P, lists, Mt, ns)
        if graphs:
            tr.capture()
        for _ in range(STEPS):
            tr.step()
        torch.cuda.synchronize()
        tr.sharded.gather_state()
        q.put((rank, tr.standard(tr.params), tr.standard(tr.m), tr.losses()['loss']))
        dist.destroy_process_group()
    except Exception as e:   # surface the error in the parent
        q.put((rank, repr(e), None, None))
        raise


@pytest.mark.parametrize('reg,graphs', [(0.0, False), (0.1, True)])
def test_sharded_dp_step_matches_single_process(reg, graphs):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29600 + (os.getpid() + int(graphs)) % 1000
    ps = [ctx.Process(target=_worker, args=(r, port, reg, graphs, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, prm, m, loss = q.get(timeout=300)
        assert m is not None, prm
        res[r] = (prm, m, loss)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    from oracle import model_ref
    lists, Mt, ns = problem(3, C, V, (20, 40, 80))
    P = model_ref.init_params(V, D, seed=3, bias_std=0.01)
    single = _make(0, 1, W * B, reg, P, lists, Mt, ns)
    for _ in range(STEPS):
        single.step()
    torch.cuda.synchronize()
    want_p, want_m = single.params.cpu().numpy(), single.m.cpu().numpy()
    for r in range(W):
        np.testing.assert_array_equal(res[r][0], res[0][0])       # ranks agree exactly
        assert rel_err(res[r][0], want_p) < 1e-5
        assert rel_err(res[r][1], want_m) < 1e-4
    assert abs(np.mean([res[r][2] for r in range(W)]) - single.losses()['loss']) < 1e-4 * single.losses()['loss']


def _shard_worker(rank, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(W), LOCAL_RANK='0', HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        import torch.distributed as dist
        from cubecobrarecommender_amd.layout import Layout
        from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer, reg_rows_for
        from oracle import model_ref
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=W)
        lists, Mt, ns = problem(3, C, V, (20, 40, 80))
        P = model_ref.init_params(V, D, seed=3, bias_std=0.01)
        lo, hi = reg_rows_for(ns, W, rank)
        cfg = TrainConfig(V=V, d=D, batch_size=B, reg=0.1, dtype='fp32', seed=3, rank=rank, world=W,
                          reg_shard=True)
        # the rank holds only its rows of M~
        data = DeviceDataset(lists, V, y_mtx=Mt[lo:hi].astype(np.float32), neg_sampler=ns,
                             reg_rows=(lo, hi))
        tr = Trainer(cfg, data, params_flat=Layout(V, D).pack(P))
        tr.set_epoch_permutations(np.random.default_rng(4).permutation(C)[None, :])
        tr.step()
        torch.cuda.synchronize()
        xs, ys, reg = tr.batch_lists()
        q.put((rank, (xs[:B], ys, reg, tr.reg_rows, tr.reg_weight, tr.standard(tr.params),
                      tr.losses()['kl'], tr.standard(tr.grads))))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e)))
        raise


def test_row_sharded_regulariser_owner_computes():
    """M~ row-sharded across ranks at equal neg_sampler mass; each rank draws its reg
    rows from its shard (bit-exact vs the Philox oracle), weights its KL by world * m_r, and the
    averaged step equals the oracle's TF-Adam step on the mean of the ranks' gradients."""
    from oracle import model_ref, noise_ref
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29400 + os.getpid() % 1000
    ps = [ctx.Process(target=_shard_worker, args=(r, port, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, payload = q.get(timeout=300)
        assert not isinstance(payload, str), payload
        res[r] = payload
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    lists, Mt, ns = problem(3, C, V, (20, 40, 80))
    P = model_ref.init_params(V, D, seed=3, bias_std=0.01)
    cdf = noise_ref.cdf_of(ns)
    from cubecobrarecommender_amd.layout import Layout
    lay = Layout(V, D)
    for r in range(W):
        xs, ys, reg, (lo, hi), wgt, _, kl_r, g_r = res[r]
        assert lo < hi and np.all((reg >= lo) & (reg < hi))
        np.testing.assert_array_equal(reg, noise_ref.philox_reg_indices(cdf, 3, 0, r * B, B, (lo, hi)))
        # the rank's own gradient (before the reduce-scatter) = the oracle's with KL weight W * m_r
        losses, Gr = model_ref.train_forward_backward(P, xs, ys, V, D, reg=0.1 * wgt, reg_idx=reg,
                                                      y_reg=Mt[reg].astype(np.float32))
        assert abs(kl_r - wgt * losses['kl']) <= 1e-4 * abs(wgt * losses['kl'])
        got = lay.unpack(g_r)
        for k in Gr:
            assert rel_err(got[k], Gr[k]) < 1e-4, (r, k, rel_err(got[k], Gr[k]))
        np.testing.assert_array_equal(res[r][5], res[0][5])        # ranks agree exactly after Adam
    assert sum(res[r][4] for r in range(W)) == pytest.approx(W)   # shard masses sum to 1
