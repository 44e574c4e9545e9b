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
