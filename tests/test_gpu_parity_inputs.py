"""GPU training step on the REFERENCE's own batches (north_star "identical inputs").

tests/golden/generator_{small,medium,bench}.npz hold the x / y / reg rows that the reference's own
``DataGenerator.__getitem__`` produced (/root/reference/src/ml/generator.py:38-103, run by
oracle/make_golden.py with the reference imported; the third batch of each file follows an
``on_epoch_end`` reshuffle).  Here each batch is written into the device batch buffers with
``Trainer.load_batch`` (F skipped for that step), the GPU step runs on it, and its losses and
gradients are compared with ``oracle.model_ref`` on exactly the same rows, then Adam is applied
on both sides (train.py:83-102).  Bars: fp32 loss 1e-4 relative (north_star) and
gradients 1e-4 relative L2; bf16 against the bf16-operand oracle: loss 2e-4, gradients 2e-2.
M~ for the 'bench' file is the oracle's (pinned against the reference's create_adjacency_matrix on
the other two files; its neg_sampler equals the reference generator's, tests/test_oracle.py).
"""
import os

import numpy as np
import pytest
import torch

from cubecobrarecommender_amd.layout import Layout
from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
from oracle import adjacency_ref, model_ref
from tests.gpu_helpers import record_errors, rel_err

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
BARS = {'fp32': (1e-4, 1e-4), 'bf16': (2e-4, 2e-2)}   # (loss, gradient) relative
# ... and ~10x the largest error observed on MI355X over these batches (r06b: fp32 loss 1.2e-7 /
# gradients 5.0e-7; bf16 loss 1.7e-6 / gradients 5.3e-3 against the bf16-operand oracle)
TIGHT = {'fp32': (1e-6, 5e-6), 'bf16': (2e-5, 2e-2)}


def _golden(name):
    g = np.load(os.path.join(GOLDEN, f'generator_{name}.npz'))
    cubes = g['cubes'].astype(np.float64)
    if name == 'bench':
        Mt = adjacency_ref.normalise(adjacency_ref.adjacency(cubes))
    else:
        Mt = np.load(os.path.join(GOLDEN, f'adjacency_{name}.npz'))['Mt']
    lists = [np.nonzero(c)[0] for c in cubes]
    return g, lists, Mt


def _trainer(lists, Mt, ns, V, d, B, reg, dtype, P, **kw):
    cfg = TrainConfig(V=V, d=d, batch_size=B, reg=reg, dtype=dtype, seed=1, **kw)
    data = DeviceDataset(lists, V, y_mtx=Mt.astype(np.float32) if reg > 0 else None, neg_sampler=ns)
    tr = Trainer(cfg, data, params_flat=Layout(V, d).pack(P))
    tr.set_epoch_permutation(np.arange(len(lists), dtype=np.int32))
    return tr


CASES = [('small', 64, 'fp32', 0.1), ('small', 64, 'fp32', 0.0), ('medium', 64, 'fp32', 0.1),
         ('medium', 128, 'bf16', 0.1), ('bench', 256, 'fp32', 0.1), ('bench', 256, 'bf16', 0.1),
         ('bench', 256, 'bf16', 0.0)]


@pytest.mark.parametrize('name,d,dtype,reg', CASES)
def test_step_on_reference_batches_matches_oracle(name, d, dtype, reg):
    g, lists, Mt = _golden(name)
    V, B = g['cubes'].shape[1], int(g['B'])
    ns = g['neg_sampler']
    P = model_ref.init_params(V, d, seed=5, bias_std=0.01)
    tr = _trainer(lists, Mt, ns, V, d, B, reg, dtype, P)
    if name == 'bench' and dtype == 'bf16':   # the bench's kernels: fused output layers, packed towers
        assert tr.fused_out and (reg == 0 or tr.fused_reg) and tr.wpack is not None
    Mo = {k: np.zeros_like(v) for k, v in P.items()}
    Vo = {k: np.zeros_like(v) for k, v in P.items()}
    mode = 'bf16' if dtype == 'bf16' else 'fp64'
    lt, gt = BARS[dtype]
    for bi in range(g['x'].shape[0]):
        xs = [np.nonzero(r)[0] for r in g['x'][bi]]
        ys = [np.nonzero(r)[0] for r in g['y'][bi]]
        reg_idx = g['reg'][bi]
        tr.load_batch(g['x'][bi], g['y'][bi], reg_idx)   # dense 0/1 rows, as Keras receives them
        tr.forward_backward()
        torch.cuda.synchronize()
        gx, gy, greg = tr.batch_lists()                  # the step consumed the reference's batch
        for b in range(B):
            assert np.array_equal(gx[b], xs[b]) and np.array_equal(gy[b], ys[b]), b
        if reg > 0:
            assert np.array_equal(greg[:B], reg_idx)
            for r in range(B):                           # x_reg: identity rows of the reg cards
                assert np.array_equal(gx[B + r], [reg_idx[r]])
        losses, grads = model_ref.train_forward_backward(
            P, xs, ys, V, d, reg=reg, reg_idx=reg_idx if reg > 0 else None,
            y_reg=Mt[reg_idx] if reg > 0 else None, mode=mode)
        got = tr.losses()
        gflat = tr.layout.unpack(tr.grads.cpu().numpy())
        e = {'loss/bce': abs(got['bce'] - losses['bce']) / losses['bce'],
             'loss/total': abs(got['loss'] - losses['loss']) / losses['loss']}
        if reg > 0:
            e['loss/kl'] = abs(got['kl'] - losses['kl']) / losses['kl']
        e.update({k: rel_err(gflat[k], grads[k]) for k in grads if reg or not k.startswith('decoder_for_reg')})
        record_errors(f'refbatch_{name}_{d}_{dtype}_{reg}', bi, e)
        bad = {k: v for k, v in e.items() if not v < (lt if k.startswith('loss/') else gt)}
        assert not bad, (bi, bad)
        tl, tg = TIGHT[dtype]
        bad = {k: v for k, v in e.items() if not v < (tl if k.startswith('loss/') else tg)}
        assert not bad, ('tight', bi, bad)
        tr.apply()
        torch.cuda.synchronize()
        P, Mo, Vo = model_ref.adam_tf(P, Mo, Vo, grads, t=bi + 1)
        got_p = tr.layout.unpack(tr.params.cpu().numpy())
        for k in ('encoder/encoded_1/kernel', 'encoder/encoded_2/kernel', 'decoder/reconstruct/kernel'):
            assert rel_err(got_p[k], P[k]) < (1e-3 if dtype == 'fp32' else 5e-2), k
        # continue both sides from the oracle's weights (Adam's sign on ~0 gradients would otherwise
        # diverge the comparison, not the arithmetic; tests/test_gpu_train.py does the same)
        tr.params.copy_(torch.from_numpy(tr.layout.pack(P)))
        tr.m.copy_(torch.from_numpy(tr.layout.pack(Mo)))
        tr.v.copy_(torch.from_numpy(tr.layout.pack(Vo)))
        tr.refresh_shadow()


@pytest.mark.parametrize('reg', [0.0, 0.1])
def test_bench_config_on_reference_batches(reg):
    """bench.py's own TrainConfig (W1's Adam in its gradient kernel, the output layers' Adam tails
    beside the tower chains, F prefetched in the Adam launch — which load_batch overrides) on the
    reference's batches: losses per step at the bf16 bar and the updated parameters against the
    oracle's Adam trajectory; the following step() without a host batch draws F again."""
    g, lists, Mt = _golden('bench')
    V, B, d = g['cubes'].shape[1], int(g['B']), 256
    ns = g['neg_sampler']
    P = model_ref.init_params(V, d, seed=5, bias_std=0.01)
    tr = _trainer(lists, Mt, ns, V, d, B, reg, 'bf16', P, fuse_w1_adam=True, wo_adam_in_tower=True)
    assert tr.fuse_w1 and tr.wo_ranges is not None and tr.prefetch
    Mo = {k: np.zeros_like(v) for k, v in P.items()}
    Vo = {k: np.zeros_like(v) for k, v in P.items()}
    for bi in range(g['x'].shape[0]):
        xs = [np.nonzero(r)[0] for r in g['x'][bi]]
        ys = [np.nonzero(r)[0] for r in g['y'][bi]]
        reg_idx = g['reg'][bi]
        tr.load_batch(xs, ys, reg_idx)                   # index lists this time
        tr.step()
        tr.flush()
        torch.cuda.synchronize()
        losses, grads = model_ref.train_forward_backward(
            P, xs, ys, V, d, reg=reg, reg_idx=reg_idx if reg > 0 else None,
            y_reg=Mt[reg_idx] if reg > 0 else None, mode='bf16')
        got = tr.losses()
        e = {'loss/total': abs(got['loss'] - losses['loss']) / losses['loss']}
        P, Mo, Vo = model_ref.adam_tf(P, Mo, Vo, grads, t=bi + 1)
        got_p = tr.layout.unpack(tr.params.cpu().numpy())
        e.update({f'param/{k}': rel_err(got_p[k], P[k]) for k in
                  ('encoder/encoded_1/kernel', 'decoder/reconstruct/kernel', 'decoder/reconstruct/bias')})
        record_errors(f'refbatch_benchcfg_{reg}', bi, e)
        assert e['loss/total'] < BARS['bf16'][0], e
        assert all(v < 5e-2 for k, v in e.items() if k.startswith('param/')), e
        tr.params.copy_(torch.from_numpy(tr.layout.pack(P)))
        tr.m.copy_(torch.from_numpy(tr.layout.pack(Mo)))
        tr.v.copy_(torch.from_numpy(tr.layout.pack(Vo)))
        tr.refresh_shadow()
    # no host batch: the next step draws its own F (the batch differs from the last host batch)
    tr.step()
    tr.flush()
    torch.cuda.synchronize()
    gx, _, _ = tr.batch_lists()
    assert any(not np.array_equal(gx[b], np.nonzero(g['x'][-1][b])[0]) for b in range(B))
    tr.check_status()
