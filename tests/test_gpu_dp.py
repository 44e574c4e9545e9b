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
