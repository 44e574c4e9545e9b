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


# the bench's shape class: bf16, d = 256, B = 128 per rank — fused D1 output kernel, packed tower
# and D3 images, MFMA W1 gradient — the kernels the 8-GPU bench runs
SHAPES = {'small': dict(V=700, d=64, B=32, C=256, dtype='fp32'),
          'bench': dict(V=2500, d=256, B=128, C=1024, dtype='bf16')}


def _make(rank, world, batch, reg, P, lists, Mt, ns, shape='small', reg_shard=False):
    from cubecobrarecommender_amd.layout import Layout
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    S = SHAPES[shape]
    cfg = TrainConfig(V=S['V'], d=S['d'], batch_size=batch, reg=reg, dtype=S['dtype'], seed=3, rank=rank,
                      world=world, reg_shard=reg_shard)
    data = DeviceDataset(lists, S['V'], y_mtx=Mt.astype(np.float32) if reg else None, neg_sampler=ns)
    tr = Trainer(cfg, data, params_flat=Layout(S['V'], S['d']).pack(P))
    tr.set_epoch_permutations(np.random.default_rng(4).permutation(S['C'])[None, :])
    return tr


def _problem(shape):
    from oracle import model_ref
    S = SHAPES[shape]
    lists, Mt, ns = problem(3, S['C'], S['V'], (20, 40, 80))
    P = model_ref.init_params(S['V'], S['d'], seed=3, bias_std=0.01)
    return lists, Mt, ns, P


def _worker(rank, port, reg, graphs, q, shape='small', reg_shard=False):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(W), LOCAL_RANK='0', HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=W)
        lists, Mt, ns, P = _problem(shape)
        tr = _make(rank, W, SHAPES[shape]['B'], reg, P, lists, Mt, ns, shape, reg_shard=reg_shard)
        assert tr.owner == (reg_shard and reg > 0)
        if shape == 'bench':
            assert tr.fused_out and tr.wpack is not None and tr.gpre1p is not None
        if graphs:
            tr.capture()
        for _ in range(STEPS):
            tr.step()
        torch.cuda.synchronize()
        tr.sharded.gather_state()
        tr.check_status()
        extra = (tr.reg_idx.cpu().numpy(), tr.reg_rows, tr.Breg) if tr.owner else None
        q.put((rank, tr.standard(tr.params), tr.standard(tr.m), tr.losses()['loss'], extra))
        dist.destroy_process_group()
    except Exception as e:   # surface the error in the parent
        q.put((rank, repr(e), None, None))
        raise


@pytest.mark.parametrize('reg,graphs,shape,reg_shard', [
    (0.0, False, 'small', False), (0.1, True, 'small', False), (0.1, False, 'small', True),
    (0.0, True, 'bench', False), (0.1, True, 'bench', False), (0.1, True, 'bench', True)])
def test_sharded_dp_step_matches_single_process(reg, graphs, shape, reg_shard):
    """Two ranks of B == one process of 2B (same cubes, F draws, regulariser draws and averaged
    gradients).  reg_shard: M~ row-sharded, owner computes — every rank draws the
    2B global reg rows and keeps the ones in its shard, so the step is still the one-process step."""
    from oracle import noise_ref
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29600 + (os.getpid() + int(graphs) + 7 * len(shape) + 3 * int(reg_shard)) % 1000
    ps = [ctx.Process(target=_worker, args=(r, port, reg, graphs, q, shape, reg_shard)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, prm, m, loss, extra = q.get(timeout=300)
        assert m is not None, prm
        res[r] = (prm, m, loss, extra)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    lists, Mt, ns, P = _problem(shape)
    single = _make(0, 1, W * SHAPES[shape]['B'], reg, P, lists, Mt, ns, shape)
    if graphs:
        single.capture()
    for _ in range(STEPS):
        single.step()
    torch.cuda.synchronize()
    single.flush()
    want_p, want_m = single.params.cpu().numpy(), single.m.cpu().numpy()
    bf16 = SHAPES[shape]['dtype'] == 'bf16'
    for r in range(W):
        np.testing.assert_array_equal(res[r][0], res[0][0])       # ranks agree exactly
        # bf16: Adam's m/(sqrt(v)+eps) turns summation-order noise on ~0 gradients into whole
        # +-lr steps on those elements (the oracle tests re-sync for the same reason)
        assert rel_err(res[r][0], want_p) < (2e-4 if bf16 else 1e-5)
        assert rel_err(res[r][1], want_m) < (2e-3 if bf16 else 1e-4)
    assert abs(np.mean([res[r][2] for r in range(W)]) - single.losses()['loss']) < 1e-4 * single.losses()['loss']
    if reg_shard and reg > 0:   # the owned rows of the last step's global draws, per the oracle
        B = SHAPES[shape]['B']
        cdf = noise_ref.cdf_of(ns)
        for r in range(W):
            idx, (lo, hi), cap = res[r][3]
            want, n, over = noise_ref.owner_reg_rows(cdf, 3, STEPS - 1, W * B, lo, hi, cap)
            assert not over and n > 0
            np.testing.assert_array_equal(idx, want)


def _cli_worker(rank, port, out_dir, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(W), LOCAL_RANK='0', HSA_ENABLE_IPC_MODE_LEGACY='0',
                      CCREC_DIST_BACKEND='gloo')
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'scripts'))
        import train as train_cli
        model = train_cli.main(['2', '32', 'dp_ckpt', '0.1', '0.2', '0', '--synthetic', '256', '1500',
                                '--d', '64', '--out-dir', out_dir])
        q.put((rank, model._current_flat(), model._m))
    except Exception as e:
        q.put((rank, repr(e), None))
        raise


def test_train_cli_two_ranks_saves_checkpoint(tmp_path):
    """scripts/train.py under two ranks (rank 0's save used to enter collectives the
    other rank never joined): fit gathers the sharded Adam state on every rank, rank 0 writes
    ml_files/<name>/, and the checkpoint loads back with the trained weights and moments."""
    from cubecobrarecommender_amd.model import load_model
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29300 + os.getpid() % 1000
    ps = [ctx.Process(target=_cli_worker, args=(r, port, str(tmp_path), q)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, flat, m = q.get(timeout=300)
        assert m is not None, flat
        res[r] = (flat, m)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    m2 = load_model(str(tmp_path / 'dp_ckpt'))
    np.testing.assert_array_equal(m2._current_flat(), res[0][0])
    np.testing.assert_array_equal(m2._m, res[0][1])
    assert m2._step == 2 * (256 // (32 * W))
