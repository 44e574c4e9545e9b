"""CPU tests of host-side logic (no GPU)."""
import numpy as np

from cubecobrarecommender_amd.synthetic import neg_sampler_from_csr
from oracle import adjacency_ref, noise_ref
from tests.gpu_helpers import synthetic_lists


def test_neg_sampler_closed_form_matches_dense_definition():
    rng = np.random.default_rng(0)
    V = 400
    lists = synthetic_lists(rng, 150, V, sizes=(5, 30, 80), never_seen=7)
    Mt = adjacency_ref.normalise(adjacency_ref.adjacency_from_lists(lists, V))
    want = noise_ref.neg_sampler_of(Mt)
    indptr = np.zeros(len(lists) + 1, np.int64)
    indptr[1:] = np.cumsum([len(l) for l in lists])
    got = neg_sampler_from_csr(indptr, np.concatenate(lists), V)
    assert np.max(np.abs(got - want) / want) < 1e-12


def test_reg_row_shards_equal_mass_and_owner_draws():
    """M~ row shards at equal cumulative neg_sampler mass; a rank's reg draws (Philox
    oracle, shard-conditioned) stay in its rows and follow neg_sampler restricted to them."""
    import pytest
    from cubecobrarecommender_amd.trainer import reg_row_shards
    rng = np.random.default_rng(5)
    V = 3000
    ns = 1.0 / (1.0 + rng.permutation(V))
    ns /= ns.sum()
    cdf = np.cumsum(ns)
    cdf /= cdf[-1]
    for W in (1, 2, 4, 8):
        b, m = reg_row_shards(cdf, W)
        assert b[0] == 0 and b[-1] == V and np.all(np.diff(b) > 0)
        assert abs(m.sum() - 1.0) < 1e-12
        assert np.all(np.abs(m - 1.0 / W) < ns.max() + 1e-12)   # off by at most one card's mass
    b, m = reg_row_shards(cdf, 4)
    for r in range(4):
        lo, hi = int(b[r]), int(b[r + 1])
        draws = noise_ref.philox_reg_indices(cdf, 11, 0, 0, 40000, (lo, hi))
        assert draws.min() >= lo and draws.max() < hi
        freq = np.bincount(draws - lo, minlength=hi - lo) / len(draws)
        want = ns[lo:hi] / ns[lo:hi].sum()
        top = np.argsort(-want)[:20]
        assert np.all(np.abs(freq[top] - want[top]) < 5 * np.sqrt(want[top] / len(draws)) + 1e-3)
    # unsharded oracle path unchanged by the new argument
    np.testing.assert_array_equal(noise_ref.philox_reg_indices(cdf, 11, 3, 7, 500),
                                  noise_ref.philox_reg_indices(cdf, 11, 3, 7, 500, None))
    heavy = np.full(10, 0.01)
    heavy[0] = 0.91
    with pytest.raises(ValueError):
        reg_row_shards(np.cumsum(heavy) / heavy.sum(), 4)
