"""GPU parity of the co-occurrence graph (csrc/cooccur.hip) through the C-ABI.

Pinned against the reference's own create_adjacency_matrix output (tests/golden/adjacency_*.npz,
made by tests/golden/make_golden.py from src/non_ml/utils.py:75-91 and src/ml/train.py:69-71):
M (f64) and the integer counts are bit-exact; M~ (f32) is compared with the f32 rounding of the
reference's f64 M~ to at most 1 ulp (the reference divides by an f64 pairwise row sum, the
kernel by the exact integer row sum — the two round apart only at f32 midpoints).
"""
import numpy as np
import pytest
import torch

from oracle import adjacency_ref
from tests.gpu_helpers import synthetic_lists

pytestmark = pytest.mark.gpu


def _csr(lists):
    indptr = np.zeros(len(lists) + 1, np.int64)
    indptr[1:] = np.cumsum([len(x) for x in lists])
    idx = np.concatenate([np.asarray(x, np.int64) for x in lists]) if lists else np.zeros(0, np.int64)
    return indptr, idx


def _dense(lists, V):
    X = np.zeros((len(lists), V), np.float64)
    for c, x in enumerate(lists):
        X[c, np.asarray(x, np.int64)] = 1
    return X


def _ulp_diff(a32, b32):
    a = np.asarray(a32, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b32, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def _check_all(lists, V, chunk=0, force_diag=None, with_counts=True):
    from cubecobrarecommender_amd.adjacency import adjacency_gpu
    indptr, idx = _csr(lists)
    outs = ('counts', 'M', 'Mt') if with_counts else ('M', 'Mt')
    got = adjacency_gpu(indptr, idx, V, outs, force_diag=force_diag, chunk_cubes=chunk)
    torch.cuda.synchronize()
    X = _dense(lists, V)
    if with_counts:
        counts = (X.T @ X).astype(np.int64)
        np.testing.assert_array_equal(got['counts'].cpu().numpy(), counts)
    M = adjacency_ref.adjacency(X, force_diag=force_diag)
    np.testing.assert_array_equal(got['M'].cpu().numpy(), M)
    Mt = adjacency_ref.normalise(adjacency_ref.adjacency(X)).astype(np.float32)
    assert _ulp_diff(got['Mt'].cpu().numpy(), Mt).max() <= 1
    return got


@pytest.mark.parametrize('name', ['small', 'medium'])
def test_adjacency_matches_reference_golden(golden_dir, name):
    from cubecobrarecommender_amd.adjacency import create_adjacency_matrix, dense_to_csr, adjacency_gpu
    g = np.load(f'{golden_dir}/adjacency_{name}.npz')
    cubes = g['cubes']
    M = create_adjacency_matrix(cubes)                      # the reference's call shape
    assert M.dtype == np.float64
    np.testing.assert_array_equal(M, g['M'])                # bit-exact vs utils.create_adjacency_matrix
    indptr, idx = dense_to_csr(cubes)
    Mt = adjacency_gpu(indptr, idx, cubes.shape[1], ('Mt',))['Mt'].cpu().numpy()
    assert _ulp_diff(Mt, g['Mt'].astype(np.float32)).max() <= 1
    np.testing.assert_allclose(Mt, g['Mt'], rtol=1.2e-7, atol=0)


@pytest.mark.parametrize('V,C', [(1, 3), (5, 7), (130, 40), (301, 257), (700, 300), (1029, 611)])
def test_adjacency_random(V, C):
    rng = np.random.default_rng(V * 7 + C)
    lists = synthetic_lists(rng, C, V, sizes=(1, min(V, 3), min(V, 25), min(V, 90)),
                            never_seen=min(3, V - 1))
    _check_all(lists, V)


def test_adjacency_duplicates_empty_cubes_and_unseen_cards():
    V = 203
    rng = np.random.default_rng(11)
    lists = []
    for c in range(150):
        n = int(rng.integers(0, 30))
        x = rng.integers(0, V - 20, size=n)          # cards >= V-20 never appear
        if c % 5 == 0 and n:
            x = np.concatenate([x, x[: n // 2]])      # repeated ids collapse (cubes[c, ids] = 1)
        lists.append(rng.permutation(x))
    lists[7] = np.zeros(0, np.int64)
    got = _check_all(lists, V)
    Mt = got['Mt'].cpu().numpy()
    for j in range(V - 20, V):                        # unseen card: M row 0, M~ row e_j
        assert not got['M'][j].any()
        np.testing.assert_array_equal(Mt[j], np.eye(V, dtype=np.float32)[j])


def test_adjacency_no_cubes():
    from cubecobrarecommender_amd.adjacency import adjacency_gpu
    got = adjacency_gpu(np.zeros(1, np.int64), np.zeros(0, np.int64), 9, ('counts', 'M', 'Mt'))
    assert not got['counts'].any() and not got['M'].any()
    np.testing.assert_array_equal(got['Mt'].cpu().numpy(), np.eye(9, dtype=np.float32))


def test_adjacency_force_diag():
    rng = np.random.default_rng(5)
    lists = synthetic_lists(rng, 60, 150, sizes=(5, 20))
    _check_all(lists, 150, force_diag=0.0)
    _check_all(lists, 150, force_diag=2.5)


@pytest.mark.parametrize('with_counts', [True, False])
def test_adjacency_chunked_cubes(with_counts):
    """Cubes in chunks (bounded Xt): partial counts accumulate, results identical."""
    rng = np.random.default_rng(9)
    lists = synthetic_lists(rng, 700, 517, sizes=(10, 40, 120))
    _check_all(lists, 517, chunk=128, with_counts=with_counts)
    _check_all(lists, 517, chunk=300, with_counts=with_counts)


def test_adjacency_rejects_bad_ids():
    from cubecobrarecommender_amd.adjacency import adjacency_gpu
    with pytest.raises(IndexError):
        adjacency_gpu(np.array([0, 2]), np.array([1, 10]), 10)


def test_adjacency_full_size_properties():
    """BASELINE-scale graph (|V| = 22000, 16384 synthetic cubes of 180-720 cards): exact
    integer identities that hold at any size — symmetric counts, diag = per-card cube counts,
    row sums = S_i — plus M = counts/diag and M~ = counts/rowsum on sampled rows."""
    from cubecobrarecommender_amd.adjacency import adjacency_gpu
    V, C = 22000, 16384
    rng = np.random.default_rng(1)
    pop = 1.0 / (1.0 + rng.permutation(V - 50)) ** 0.8
    sizes = rng.integers(180, 721, size=C)
    lists = []
    for n in sizes:
        g = np.log(pop) + rng.gumbel(size=V - 50)
        lists.append(np.argpartition(-g, n)[:n])
    indptr, idx = _csr(lists)
    got = adjacency_gpu(indptr, idx, V, ('counts', 'M', 'Mt'))
    cnt = got['counts']
    assert torch.equal(cnt, cnt.t())
    d = np.bincount(idx, minlength=V)
    np.testing.assert_array_equal(torch.diagonal(cnt).cpu().numpy(), d)
    S = np.bincount(idx, weights=np.repeat(sizes, sizes), minlength=V).astype(np.int64)
    np.testing.assert_array_equal(cnt.sum(1, dtype=torch.int64).cpu().numpy(), S)
    rows = rng.choice(V, 64, replace=False)
    c = cnt[rows].cpu().numpy().astype(np.float64)
    M = got['M'][rows].cpu().numpy()
    dd = d[rows].astype(np.float64)[:, None]
    np.testing.assert_array_equal(M, np.where(dd != 0, c / np.where(dd == 0, 1, dd), c))
    Mt = got['Mt'][rows].cpu().numpy()
    ss = S[rows].astype(np.float64)[:, None]
    want = np.where(ss != 0, c / np.where(ss == 0, 1, ss), np.eye(V)[rows]).astype(np.float32)
    np.testing.assert_array_equal(Mt, want)
