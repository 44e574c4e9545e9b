"""GPU recommend path vs the pinned-order CPU oracle: probabilities and top-N BIT-EXACT."""
import numpy as np
import pytest
import torch

from cubecobrarecommender_amd.layout import Layout
from cubecobrarecommender_amd.recommender import Recommender
from oracle import infer_ref, model_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def model():
    V, d = 20884, 512          # the reference checkpoint's architecture
    P = model_ref.init_params(V, d, seed=20250301, bias_std=0.01)
    rec = Recommender(Layout(V, d).pack(P), V, d)
    return V, d, P, rec


@pytest.mark.parametrize('n', [0, 1, 45, 360, 540, 720])
def test_recommend_bit_exact(model, n):
    V, d, P, rec = model
    rng = np.random.default_rng(n)
    cube = rng.choice(V, n, replace=False)
    want_p = infer_ref.recommend_probs(P, cube)
    for amount in (100, 30000, 0):
        adds, _ = infer_ref.top_n(want_p, cube, amount)
        for full, direct in ((False, False), (True, False), (False, True)):
            # graph-replayed request / + full ranking / direct (uncaptured) launch sequence
            saved = rec.cap
            if direct:
                rec._graph_handle()
                rec.cap = -1
            try:
                out = rec.recommend(cube, amount, want_probs=True, want_order=full)
            finally:
                rec.cap = saved
            assert np.array_equal(out['probs'], want_p)                   # bit-exact fp32
            if full:
                assert np.array_equal(out['order'], infer_ref.rank(want_p))
            assert np.array_equal(out['additions'], adds)
            assert np.array_equal(out['add_vals'], want_p[adds])
            assert np.array_equal(out['cut_vals'], want_p[cube])


def test_ties_rank_higher_index_first(model):
    V, d, P, rec = model
    # saturate the output: huge bias makes many probabilities exactly 1.0f
    P2 = dict(P)
    P2['decoder/reconstruct/bias'] = np.where(np.arange(V) % 3 == 0, 40.0, -3.0).astype(np.float32)
    r2 = Recommender(Layout(V, d).pack(P2), V, d)
    cube = np.arange(0, 300, 7)
    fast = r2.recommend(cube, 20000)
    out = r2.recommend(cube, 200, want_probs=True, want_order=True)
    want_p = infer_ref.recommend_probs(P2, cube)
    assert np.array_equal(out['probs'], want_p)
    assert np.sum(want_p == 1.0) > 100
    assert np.array_equal(out['order'], infer_ref.rank(want_p))
    top = out['order'][:50]
    assert np.all(np.diff(top) < 0)    # equal 1.0f values: higher index first
    assert np.array_equal(fast['additions'], infer_ref.top_n(want_p, cube, 20000)[0])


def test_encoder_decoder_batch(model):
    V, d, P, rec = model
    rng = np.random.default_rng(1)
    lists = [rng.choice(V, k, replace=False) for k in (10, 200, 0, 500)]
    z = rec.encode_lists(lists).cpu().numpy()
    for r, l in enumerate(lists):
        assert np.array_equal(z[r], infer_ref.encode32(P, l))
    p = rec.decode(torch.from_numpy(z)).cpu().numpy()
    for r in range(len(lists)):
        assert np.array_equal(p[r], infer_ref.decode32(P, z[r]))


def _topn(probs, cube, amount, want_order=True):
    from cubecobrarecommender_amd import _lib as L
    V = probs.numel()
    dev = probs.device
    n = len(cube)
    ci = torch.tensor(np.asarray(cube, np.int32), device=dev) if n else torch.zeros(1, dtype=torch.int32, device=dev)
    want = min(max(amount, 1), V)
    adds = torch.full((want,), -7, dtype=torch.int32, device=dev)
    addv = torch.zeros(want, device=dev)
    cutv = torch.zeros(max(n, 1), device=dev)
    nadd = torch.zeros(1, dtype=torch.int32, device=dev)
    order = torch.zeros(V, dtype=torch.int32, device=dev)
    ws = torch.zeros(int(L.lib().cc_topn_workspace_size(V)) // 4 + 1, dtype=torch.int32, device=dev)
    L.call('cc_topn', L.ptr(probs), V, L.ptr(ci), n, amount, L.ptr(adds), L.ptr(nadd), L.ptr(addv), L.ptr(cutv),
           L.ptr(order) if want_order else None, L.ptr(ws), L.stream_ptr())
    torch.cuda.synchronize()
    k = int(nadd.item())
    return adds[:k].cpu().numpy(), addv[:k].cpu().numpy(), cutv[:n].cpu().numpy(), order.cpu().numpy()


@pytest.mark.parametrize('V', [1, 63, 700, 4097, 20884, 22000, 22803, 30001, 60000])
def test_topn_kernels_bit_exact(V):
    """Tiled request path (order=NULL) and the single-workgroup full ranking vs the pinned stable
    ranking, with heavy ties, zero probabilities, 1 and many tiles, partial last tiles."""
    rng = np.random.default_rng(V)
    vals = rng.random(V).astype(np.float32)
    vals[rng.random(V) < 0.3] = np.float32(0.25)          # tie block
    vals[rng.random(V) < 0.05] = np.float32(0.0)
    probs = torch.from_numpy(vals).cuda()
    n = min(V, 3 + V // 40)
    cube = np.sort(rng.choice(V, n, replace=False))
    want_order = infer_ref.rank(vals)
    for full in (False, True):
        for amount in (0, 5, 100, V + 10):
            adds, addv, cutv, order = _topn(probs, cube, amount, want_order=full)
            exp_adds, _ = infer_ref.top_n(vals, cube, amount)
            if full:
                assert np.array_equal(order, want_order), amount
            assert np.array_equal(adds, exp_adds), (full, amount)
            assert np.array_equal(addv, vals[exp_adds])
            assert np.array_equal(cutv, vals[cube])


def test_topn_unaligned_probs():
    V = 2000
    vals = np.random.default_rng(3).random(V + 1).astype(np.float32)
    buf = torch.from_numpy(vals).cuda()
    probs = buf[1:]                                          # 4-byte aligned only
    adds, _, _, order = _topn(probs, [5, 9], 50)
    assert np.array_equal(order, infer_ref.rank(vals[1:]))
    assert np.array_equal(adds, infer_ref.top_n(vals[1:], [5, 9], 50)[0])
    adds, _, _, _ = _topn(probs, [5, 9], 3000, want_order=False)
    assert np.array_equal(adds, infer_ref.top_n(vals[1:], [5, 9], 3000)[0])


@pytest.mark.parametrize('V,d', [(700, 64), (1001, 128), (4000, 1024)])
def test_recommend_other_shapes(V, d):
    P = model_ref.init_params(V, d, seed=V, bias_std=0.01)
    rec = Recommender(Layout(V, d).pack(P), V, d)
    rng = np.random.default_rng(d)
    for n in (0, 1, 33, min(V, 500)):
        cube = rng.choice(V, n, replace=False)
        want_p = infer_ref.recommend_probs(P, cube)
        out = rec.recommend(cube, 40, want_probs=True, want_order=True)
        assert np.array_equal(out['probs'], want_p)
        assert np.array_equal(out['order'], infer_ref.rank(want_p))
        assert np.array_equal(out['additions'], infer_ref.top_n(want_p, cube, 40)[0])
        out = rec.recommend(cube, V, want_probs=False)
        assert np.array_equal(out['additions'], infer_ref.top_n(want_p, cube, V)[0])
        assert np.array_equal(out['cut_vals'], want_p[cube])
