"""GPU test of the data-parallel training step end to end: two ranks (two processes on the one
GPU, gloo for the collectives) run Trainer.step() — bucketed reduce-scatter overlapped with the
towers' backward, Adam on each rank's shard, all-gathered parameters (zero.py) — eagerly and as
graph replays, and must match one process training on the concatenated batch."""
import os
import queue

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.gpu_helpers import problem, progress, rel_err

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
    import faulthandler
    faulthandler.dump_traceback_later(170, exit=True)   # a stuck child names where it is stuck
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
        if shape == 'bench':   # the output layers' all-gather runs at the next step's head (zero.py)
            assert tr.sharded.defer_out
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
    (0.0, True, 'bench', False), (0.1, True, 'bench', False), (0.1, True, 'bench', True),
    (0.0, False, 'bench', False)])
def test_sharded_dp_step_matches_single_process(reg, graphs, shape, reg_shard):
    """Two ranks of B == one process of 2B (same cubes, F draws, regulariser draws and averaged
    gradients).  reg_shard: M~ row-sharded, owner computes — every rank draws the
    2B global reg rows and keeps the ones in its shard, so the step is still the one-process step.
    The bench shape defers the output layers' all-gather to the next step's head (zero.py): before
    the phase graphs (graphs) or at the forward's hook_d1 (eager launches)."""
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


# ---------------------------------------------------------------------------------------------
# bench.py's exact data-parallel configuration (VERDICT r2 "make the code the 8-GPU run will
# execute actually run"): |V| = 22,000, d = 256, B = 512 per rank, bf16, reg 0.1, M~ row-sharded
# (owner computes), captured graphs, 3 steps.  Two ranks share the one GPU over gloo, so zero.py
# runs reduce_scatter_tensor / all_gather_into_tensor (host-staged) — the calls RCCL runs.
BENCH_DP = dict(V=22000, d=256, B=512, C=4096, reg=0.1, seed=1234, steps=3)


def _bench_problem():
    from cubecobrarecommender_amd.synthetic import neg_sampler_from_csr, synthetic_cubes
    S = BENCH_DP
    indptr_t, indices_t = synthetic_cubes(S['C'], S['V'], seed=20250301, device='cuda')
    indptr, indices = np.asarray(indptr_t), np.asarray(indices_t)
    return indptr, indices, neg_sampler_from_csr(indptr, indices, S['V'])


def _bench_trainer(rank, world, batch, reg_shard, fuse_w1_adam=True):
    from cubecobrarecommender_amd.adjacency import adjacency_normalised_gpu
    from cubecobrarecommender_amd.layout import glorot_flat
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer, reg_rows_for
    S = BENCH_DP
    indptr, indices, ns = _bench_problem()
    y = adjacency_normalised_gpu(indptr, indices, S['V'], device='cuda')
    rows = None
    if reg_shard:   # as bench.py: keep only this rank's rows of M~
        rows = reg_rows_for(ns, world, rank)
        y = y[rows[0]:rows[1]].clone()
    data = DeviceDataset(csr=(indptr, indices), num_cards=S['V'], neg_sampler=ns, y_mtx=y, device='cuda',
                         reg_rows=rows)
    cfg = TrainConfig(V=S['V'], d=S['d'], batch_size=batch, reg=S['reg'], dtype='bf16', seed=S['seed'],
                      rank=rank, world=world, reg_shard=reg_shard, fuse_w1_adam=fuse_w1_adam)
    tr = Trainer(cfg, data, params_flat=glorot_flat(S['V'], S['d'], seed=42))
    perm = np.random.default_rng(99).permutation(S['C']).astype(np.int32)
    tr.set_epoch_permutations(perm[None, :])
    return tr, perm, (indptr, indices, ns)


def _bench_worker(rank, port, q):
    import faulthandler
    faulthandler.dump_traceback_later(170, exit=True)   # a stuck child names where it is stuck
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(W), LOCAL_RANK='0', HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=W)
        tr, _, _ = _bench_trainer(rank, W, BENCH_DP['B'], True)
        assert tr.owner and tr.fused_out and tr.fused_reg and not tr.fuse_w1
        tr.capture()
        losses = []
        for _ in range(BENCH_DP['steps']):
            tr.step()
            torch.cuda.synchronize()
            losses.append(tr.losses())
        tr.sharded.gather_state()
        tr.check_status()
        q.put((rank, tr.standard(tr.params), tr.standard(tr.m), losses))
        dist.destroy_process_group()
    except Exception as e:   # surface the error in the parent
        q.put((rank, repr(e), None, None))
        raise


@pytest.mark.timeout(600)
def test_bench_dp_configuration_matches_single_process_and_oracle():
    """Two ranks of bench.py's DP Trainer == one process of B = 1,024 on the same global draws
    (parameters and Adam m after 3 steps, per-step mean loss), and that process's first step
    against the bf16-emulating oracle (losses and gradients)."""
    from oracle import model_ref, noise_ref
    from cubecobrarecommender_amd.layout import Layout
    from tests.gpu_helpers import record_errors
    S = BENCH_DP
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29900 + os.getpid() % 97
    ps = [ctx.Process(target=_bench_worker, args=(r, port, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, prm, m, losses = q.get(timeout=500)
        assert m is not None, prm
        res[r] = (prm, m, losses)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    # (unfused W1 Adam so the step's W1 gradient is stored for the oracle comparison)
    single, perm, (indptr, indices, ns) = _bench_trainer(0, 1, W * S['B'], False, fuse_w1_adam=False)
    P0 = Layout(S['V'], S['d']).unpack(single.standard(single.params))
    single.capture()
    want_losses = []
    for step in range(S['steps']):
        single.step()
        torch.cuda.synchronize()
        want_losses.append(single.losses())
        if step == 0:
            g0 = single.layout.unpack(single.standard(single.grads))
            l0 = dict(want_losses[0])
    single.flush()
    want_p, want_m = single.params.cpu().numpy(), single.m.cpu().numpy()
    np.testing.assert_array_equal(res[0][0], res[1][0])         # ranks agree exactly
    ep = rel_err(res[0][0], want_p)
    em = rel_err(res[0][1], want_m)
    el = [abs(np.mean([res[r][2][s]['loss'] for r in range(W)]) - want_losses[s]['loss']) / want_losses[s]['loss']
          for s in range(S['steps'])]
    record_errors('bench_dp_vs_single', S['steps'], {'params': ep, 'm': em, **{f'loss{s}': v for s, v in enumerate(el)}})
    # ~3x the observed (r03p): params 3.8e-5, m 1.5e-3 (Adam moments of ~0 gradients); loss 1e-7
    # (r04j: the KL as sum t ln t - sum t ln p, two sums of ~10x the KL's size, in per-lane fp32
    # partials over the ranks' and the one process's different row groupings)
    assert ep < 1.2e-4 and em < 4.5e-3 and max(el) < 3e-7, (ep, em, el)
    # the one-process step 0 against the oracle (bf16 operands emulated)
    lists = [indices[indptr[c]:indptr[c + 1]] for c in range(S['C'])]
    B2 = W * S['B']
    cdf = noise_ref.cdf_of(ns)
    oxs, oys, oreg, _ = noise_ref.philox_noise_batch([lists[c] for c in perm[:B2]], cdf, ns, S['seed'], 0)
    from oracle import adjacency_ref
    y_reg = adjacency_ref.normalised_rows_from_lists(lists, S['V'], oreg)
    lo, go = model_ref.train_forward_backward(P0, oxs, oys, S['V'], S['d'], reg=S['reg'], reg_idx=oreg,
                                              y_reg=y_reg, mode='bf16')
    errs = {'loss/bce': abs(l0['bce'] - lo['bce']) / lo['bce'], 'loss/kl': abs(l0['kl'] - lo['kl']) / lo['kl']}
    errs.update({k: rel_err(g0[k], go[k]) for k in go})
    record_errors('bench_dp_single_vs_oracle', 0, errs)
    # ~3x the observed (r03p): loss 5.5e-7, gradients 7.9e-4
    assert errs['loss/bce'] < 2e-6 and errs['loss/kl'] < 2e-6, errs
    bad = {k: v for k, v in errs.items() if not k.startswith('loss/') and not v < 2.4e-3}
    assert not bad, bad


# ---------------------------------------------------------------------------------------------
# The RCCL branch (VERDICT r3 "run the code the 8-GPU run will execute"): one process drives the
# data-parallel step through a 1-rank RCCL ("nccl") process group — zero.py's reduce_scatter_tensor,
# in-place all_gather_into_tensor and the biases' all_reduce on device tensors, the next step's F
# beside the exchange (cc_noise_next), and the whole step (collectives included) captured as ONE
# hipGraph.  With one rank the shard is the whole bucket, so the step must equal the one-process
# step (different kernels for F's bit transpose, Adam and the tower images; same arithmetic).
RCCL_SHAPES = {'bench': dict(V=2500, d=256, B=128, C=1024, dtype='bf16'),
               'c5': dict(V=2500, d=1024, B=128, C=1024, dtype='fp8')}


def _rccl_trainer(shape, reg, force_dp, reg_shard, **kw):
    from cubecobrarecommender_amd.layout import Layout
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    from oracle import model_ref
    S = RCCL_SHAPES[shape]
    lists, Mt, ns = problem(5, S['C'], S['V'], (20, 40, 80))
    P = model_ref.init_params(S['V'], S['d'], seed=3, bias_std=0.01)
    cfg = TrainConfig(V=S['V'], d=S['d'], batch_size=S['B'], reg=reg, dtype=S['dtype'], seed=3,
                      force_dp=force_dp, reg_shard=reg_shard, **kw)
    data = DeviceDataset(lists, S['V'], y_mtx=Mt.astype(np.float32) if reg else None, neg_sampler=ns)
    tr = Trainer(cfg, data, params_flat=Layout(S['V'], S['d']).pack(P))
    tr.set_epoch_permutations(np.random.default_rng(4).permutation(S['C'])[None, :])
    return tr


def _rccl_run(tr, eager=2, graphed=3):
    losses = []
    for i in range(eager):
        tr.step()
        torch.cuda.synchronize()
        losses.append(tr.losses()['loss'])
        progress(f'rccl step {i} (eager, dp={tr.dp}) loss {losses[-1]}')
    tr.capture()
    progress('rccl captured')
    for i in range(graphed):
        tr.step()
        torch.cuda.synchronize()
        losses.append(tr.losses()['loss'])
        progress(f'rccl step {eager + i} (graph, dp={tr.dp}) loss {losses[-1]}')
    tr.flush()
    torch.cuda.synchronize()
    return losses


def _rccl_worker(shape, reg, reg_shard, q, chunks=0, dp_graph=True):
    os.environ.update(HSA_ENABLE_IPC_MODE_LEGACY='0')
    import faulthandler
    faulthandler.dump_traceback_later(240, exit=True)   # a stuck child names where it is stuck
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        # the process group first: RCCL's communicator before any other GPU work of this process
        progress(f'rccl {shape} reg {reg}: init_process_group')
        dist.init_process_group('nccl', store=dist.HashStore(), rank=0, world_size=1,
                                device_id=torch.device('cuda', 0))
        progress('rccl: process group up; building the DP trainer')
        tr = _rccl_trainer(shape, reg, True, reg_shard, w1_chunks=chunks, dp_graph=dp_graph)
        assert tr.dp and tr.prefetch_dp and tr.owner == (reg_shard and reg > 0)
        assert chunks == 0 or len(tr.layout.w1_chunks) == chunks
        dl = _rccl_run(tr)
        assert tr._sharded().nccl
        if dp_graph:
            assert tr.g_dp is not None, 'whole-step DP graph not captured'
        else:        # the parts path: graph replays of the phases, eager RCCL collectives between
            assert tr.g_dp is None and tr.graphs is not None
        # a replayed (or eager) step leaves its deferred output-layer all-gather pending for flush()
        tr.step()
        assert tr.sharded.out_pending == tr.sharded.defer_out
        tr.flush()
        assert not tr.sharded.out_pending
        torch.cuda.synchronize()
        dl.append(tr.losses()['loss'])
        tr.sharded.gather_state()
        tr.check_status()
        progress('rccl: DP steps done; building the one-process trainer')
        one = _rccl_trainer(shape, reg, False, False)
        assert not one.dp
        ol = _rccl_run(one)
        one.step()
        one.flush()
        torch.cuda.synchronize()
        ol.append(one.losses()['loss'])
        one.check_status()
        res = (tr.standard(tr.params), tr.standard(tr.m), tr.standard(tr.v), dl,
               one.standard(one.params), one.standard(one.m), one.standard(one.v), ol)
        del tr, one
        if not dp_graph:   # the parts path against the whole-step graph too, on the same draws
            progress('rccl: building the whole-step-graph DP trainer')
            wh = _rccl_trainer(shape, reg, True, reg_shard, w1_chunks=chunks, dp_graph=True)
            wl = _rccl_run(wh)
            assert wh.g_dp is not None
            wh.step()
            wh.flush()
            torch.cuda.synchronize()
            wl.append(wh.losses()['loss'])
            wh.sharded.gather_state()
            res = res + (wh.standard(wh.params), wh.standard(wh.m), wh.standard(wh.v), wl)
        progress('rccl: steps done; sending the result')
        q.put(res)
        dist.destroy_process_group()
        progress('rccl: process group destroyed')
    except Exception as e:   # surface the error in the parent
        import traceback
        q.put((repr(e) + traceback.format_exc(),) + (None,) * 7)
        raise


@pytest.mark.timeout(300)
@pytest.mark.parametrize('shape,reg,reg_shard,chunks,dp_graph', [
    ('bench', 0.0, False, 0, True), ('bench', 0.1, True, 0, True), ('bench', 0.1, True, 3, True),
    ('c5', 0.1, True, 0, True), ('bench', 0.0, False, 0, False), ('bench', 0.1, True, 0, False)])
def test_rccl_one_rank_dp_step_matches_one_process(shape, reg, reg_shard, chunks, dp_graph):
    """The data-parallel step over RCCL (1 rank), eager then as the captured whole-step graph
    (dp_graph) or as graph replays of its parts with eager collectives between them (not dp_graph:
    bench.py --dp-graph 0, the fallback for the multi-rank run), == the one-process step on the same
    draws: parameters, Adam moments and losses over 6 steps; the parts path also == the whole-step
    graph.  chunks: W1's gradient launched and exchanged in that many row chunks (0: the default)."""
    from tests.gpu_helpers import record_errors
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(shape, reg, reg_shard, q, chunks, dp_graph))
    p.start()
    res = None
    for _ in range(56):        # (a child that dies without a result fails the test at once)
        try:
            res = q.get(timeout=5)
            break
        except queue.Empty:
            if not p.is_alive():
                break
    assert res is not None, f'the RCCL worker exited ({p.exitcode}) without a result'
    p.join(60)
    assert res[1] is not None, res[0]
    assert p.exitcode == 0
    dp_p, dp_m, dp_v, dl, p1, m1, v1, ol = res[:8]
    errs = {'params': rel_err(dp_p, p1), 'm': rel_err(dp_m, m1), 'v': rel_err(dp_v, v1),
            'loss': max(abs(a - b) / b for a, b in zip(dl, ol)),
            'exact_params': float(np.array_equal(dp_p, p1))}
    record_errors(f'rccl1_vs_one_{shape}_{reg}_c{chunks}_g{int(dp_graph)}', 6, errs)
    if not dp_graph:
        wp, wm, wv, wl = res[8:]
        np.testing.assert_array_equal(dp_p, wp)
        np.testing.assert_array_equal(dp_m, wm)
        np.testing.assert_array_equal(dp_v, wv)
        assert list(dl) == list(wl), (dl, wl)
    # one rank: the shard is the whole bucket, the collectives are copies — the same kernels on the
    # same draws, so the step is bit-identical (observed r04: every error exactly 0)
    np.testing.assert_array_equal(dp_p, p1)
    np.testing.assert_array_equal(dp_m, m1)
    np.testing.assert_array_equal(dp_v, v1)
    assert list(dl) == list(ol), (dl, ol)


# ---------------------------------------------------------------------------------------------
# configs[4]'s step in its data-parallel form (VERDICT r3 Missing 2): d = 1024, MX-FP8 decoder
# output / regulariser GEMMs, reg 0.1, two ranks (gloo, sharing the GPU) == one process of 2B,
# with M~ replicated (the MX scale blocks along the batch rows fall on the same 32 rows) and
# row-sharded (owner computes: the regulariser branch's dW blocks group other rows, so only the
# fp8 rounding of that product differs); the one process's first step against the MX-FP8 oracle.
FP8_DP = dict(V=3000, d=1024, B=128, C=1024, reg=0.1, steps=3)


def _fp8_trainer(rank, world, batch, reg_shard):
    from cubecobrarecommender_amd.layout import Layout
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    from oracle import model_ref
    S = FP8_DP
    lists, Mt, ns = problem(9, S['C'], S['V'], (40, 80, 160))
    P = model_ref.init_params(S['V'], S['d'], seed=6, bias_std=0.01)
    cfg = TrainConfig(V=S['V'], d=S['d'], batch_size=batch, reg=S['reg'], dtype='fp8', seed=11,
                      rank=rank, world=world, reg_shard=reg_shard)
    data = DeviceDataset(lists, S['V'], y_mtx=Mt.astype(np.float32), neg_sampler=ns)
    tr = Trainer(cfg, data, params_flat=Layout(S['V'], S['d']).pack(P))
    perm = np.random.default_rng(8).permutation(S['C']).astype(np.int32)
    tr.set_epoch_permutations(perm[None, :])
    return tr, (lists, Mt, ns, P, perm)


def _fp8_worker(rank, port, reg_shard, q):
    import faulthandler
    faulthandler.dump_traceback_later(170, exit=True)   # a stuck child names where it is stuck
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(W), LOCAL_RANK='0', HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=W)
        tr, _ = _fp8_trainer(rank, W, FP8_DP['B'], reg_shard)
        assert tr.mx8 and tr.dp and tr.owner == reg_shard
        tr.capture()
        losses = []
        for _ in range(FP8_DP['steps']):
            tr.step()
            torch.cuda.synchronize()
            losses.append(tr.losses())
        tr.sharded.gather_state()
        tr.check_status()
        q.put((rank, tr.standard(tr.params), tr.standard(tr.m), losses))
        dist.destroy_process_group()
    except Exception as e:   # surface the error in the parent
        q.put((rank, repr(e), None, None))
        raise


@pytest.mark.timeout(600)
@pytest.mark.parametrize('reg_shard', [False, True])
def test_fp8_dp_step_matches_single_process_and_oracle(reg_shard):
    from oracle import adjacency_ref, model_ref, noise_ref
    from cubecobrarecommender_amd.layout import Layout
    from tests.gpu_helpers import record_errors
    S = FP8_DP
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29700 + (os.getpid() + 13 * int(reg_shard)) % 97
    ps = [ctx.Process(target=_fp8_worker, args=(r, port, reg_shard, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, prm, m, losses = q.get(timeout=500)
        assert m is not None, prm
        res[r] = (prm, m, losses)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    single, (lists, Mt, ns, P0, perm) = _fp8_trainer(0, 1, W * S['B'], False)
    single.capture()
    want = []
    for step in range(S['steps']):
        single.step()
        torch.cuda.synchronize()
        want.append(single.losses())
        if step == 0:
            g0 = single.layout.unpack(single.standard(single.grads))
    single.flush()
    np.testing.assert_array_equal(res[0][0], res[1][0])         # ranks agree exactly
    ep = rel_err(res[0][0], single.params.cpu().numpy())
    em = rel_err(res[0][1], single.m.cpu().numpy())
    el = [abs(np.mean([res[r][2][s]['loss'] for r in range(W)]) - want[s]['loss']) / want[s]['loss']
          for s in range(S['steps'])]
    record_errors(f'fp8_dp_vs_single_shard{int(reg_shard)}', S['steps'],
                  {'params': ep, 'm': em, **{f'loss{s}': v for s, v in enumerate(el)}})
    # ~3x the observed (r04ao, deterministic kernels: the same on every box): params 3.7e-9 /
    # 5.7e-9 (replicated / row-sharded M~; sharded, the regulariser dW's MX blocks group other
    # rows), m 8.6e-8 / 8.2e-8, loss 6.4e-9 (the ranks' fp32 loss partials over 128-row groups)
    if reg_shard:
        assert ep < 1.8e-8 and em < 2.6e-7 and max(el) < 2e-8, (ep, em, el)
    else:
        assert ep < 1.2e-8 and em < 2.6e-7 and max(el) < 2e-8, (ep, em, el)
    # the one process's first step against the MX-FP8-emulating oracle
    B2 = W * S['B']
    cdf = noise_ref.cdf_of(ns)
    oxs, oys, oreg, _ = noise_ref.philox_noise_batch([lists[c] for c in perm[:B2]], cdf, ns, 11, 0)
    lo, go = model_ref.train_forward_backward(P0, oxs, oys, S['V'], S['d'], reg=S['reg'], reg_idx=oreg,
                                              y_reg=Mt[oreg], mode='mx8')
    errs = {'loss/bce': abs(want[0]['bce'] - lo['bce']) / lo['bce'],
            'loss/kl': abs(want[0]['kl'] - lo['kl']) / lo['kl']}
    errs.update({k: rel_err(g0[k], go[k]) for k in go})
    record_errors('fp8_dp_single_vs_oracle', 0, errs)
    assert errs['loss/bce'] < 1e-5 and errs['loss/kl'] < 1e-5, errs
    bad = {k: v for k, v in errs.items() if not k.startswith('loss/') and not v < 5e-3}
    assert not bad, bad
