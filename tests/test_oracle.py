"""CPU tests: the oracle is pinned against the reference's own outputs (tests/golden, produced by
oracle/make_golden.py importing /root/reference) and against published known-answer vectors."""
import os

import numpy as np
import pytest

from oracle import adjacency_ref, noise_ref, philox, detmath


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for ctr, key, want in cases:
        got = philox.philox4x32(*ctr, *key)
        assert tuple(int(g) for g in got) == want


@pytest.mark.parametrize("name", ["small", "medium"])
def test_adjacency_matches_reference(golden_dir, name):
    g = np.load(os.path.join(golden_dir, f"adjacency_{name}.npz"))
    M = adjacency_ref.adjacency(g["cubes"].astype(np.float64))
    assert np.array_equal(M, g["M"])  # bit-exact vs utils.create_adjacency_matrix
    assert np.array_equal(adjacency_ref.normalise(M), g["Mt"])
    never = np.nonzero(g["cubes"].sum(0) == 0)[0]
    assert len(never) > 0 and np.all(g["M"][never] == 0)


@pytest.mark.parametrize("name", ["small", "medium", "bench"])
def test_mt_generator_replay_matches_reference(golden_dir, name):
    g = np.load(os.path.join(golden_dir, f"generator_{name}.npz"))
    cubes = g["cubes"].astype(np.float64)
    C, V = cubes.shape
    B = int(g["B"])
    if name == "bench":   # (M not stored: the oracle's M~, whose neg_sampler must be the reference's)
        Mt = adjacency_ref.normalise(adjacency_ref.adjacency(cubes))
    else:
        Mt = np.load(os.path.join(golden_dir, f"adjacency_{name}.npz"))["Mt"]
    ns = noise_ref.neg_sampler_of(Mt)
    assert np.array_equal(ns, g["neg_sampler"])
    rs = np.random.RandomState(int(g["seed"]))
    perm = np.arange(C)
    rs.shuffle(perm)                       # generator.py:63-66 at construction
    assert np.array_equal(perm, g["perm0"])
    lists = [np.nonzero(cubes[c])[0] for c in range(C)]
    mt = noise_ref.MTNoise(rs, ns, V)
    nb = g["x"].shape[0] - 1
    for bi in range(nb + 1):
        if bi == nb:                        # on_epoch_end reshuffle, then batch 0 again
            perm = np.arange(C)
            rs.shuffle(perm)
            assert np.array_equal(perm, g["perm1"])
            sel = perm[:B]
        else:
            sel = perm[bi * B:(bi + 1) * B]
        xs, ys, reg = mt.batch([lists[c] for c in sel])
        assert np.array_equal(reg, g["reg"][bi])
        for b in range(B):
            assert np.array_equal(xs[b], np.nonzero(g["x"][bi, b])[0])
            assert np.array_equal(ys[b], np.nonzero(g["y"][bi, b])[0])


def test_detmath_accuracy():
    rng = np.random.default_rng(0)
    x = rng.uniform(-700, 700, 200000)
    assert np.max(np.abs(detmath.det_exp(x) / np.exp(x) - 1)) < 4e-15
    u = rng.uniform(0, 1, 200000) + 1e-300
    assert np.max(np.abs(detmath.det_log(u) - np.log(u))) < 2e-15 * np.max(np.abs(np.log(u)))
    t = rng.uniform(0, 1, 200000)
    assert np.max(np.abs(detmath.det_cos2pi(t) - np.cos(2 * np.pi * t))) < 4e-15
    z = rng.normal(0, 10, 100000).astype(np.float32)
    s = detmath.det_sigmoid32(z)
    ref = (1 / (1 + np.exp(-z.astype(np.float64)))).astype(np.float32)
    assert np.mean(s == ref) > 0.999


def _stats_law(draw_fn, trials):
    """Collect (k, adds-in-cube violations, add-card histogram, ycut subset) over trials."""
    ks, addh = [], None
    for t in range(trials):
        inc, x, y, k = draw_fn(t)
        incs = set(inc.tolist())
        xs, ys = set(x.tolist()), set(y.tolist())
        added = xs - incs
        cut = incs - xs
        ycut = incs - ys
        assert ycut <= cut                   # ycut drawn from the cut multiset
        assert ys <= incs
        if k is not None:
            assert len(cut) <= k and len(added) <= k
        ks.append(k)
        if addh is None:
            addh = {}
        for a in added:
            addh[a] = addh.get(a, 0) + 1
    return np.array(ks), addh


def test_philox_law_matches_reference_law():
    """Statistical parity of the counter-based F with the reference's (MT) F on one cube."""
    rng = np.random.default_rng(3)
    V = 400
    ns = rng.dirichlet(np.ones(V) * 0.5)
    cdf = noise_ref.cdf_of(ns)
    inc = np.sort(rng.choice(V, 60, replace=False))
    rs = np.random.RandomState(5)
    mt = noise_ref.MTNoise(rs, ns, V)
    T = 3000

    def mt_draw(t):
        x, y = mt.cube(inc)
        return inc, x, y, None

    def ph_draw(t):
        x, y, k = noise_ref.philox_cube(inc, cdf, ns, seed=11, step=t, slot=0)
        return inc, x, y, k

    # k distribution: compare the number of distinct cut cards (observable on both)
    k_mt, h_mt = _stats_law(mt_draw, T)
    k_ph, h_ph = _stats_law(ph_draw, T)
    def ncut(draw):
        return np.array([len(set(inc.tolist()) - set(draw(t)[1].tolist())) for t in range(T)])
    a, b = ncut(mt_draw), ncut(ph_draw)
    assert abs(a.mean() - b.mean()) < 4 * np.sqrt(a.var() / T + b.var() / T)
    # added-card frequencies follow neg_sampler restricted to the excludes
    ex = np.setdiff1d(np.arange(V), inc)
    p = ns[ex] / ns[ex].sum()
    top = ex[np.argsort(-p)[:20]]
    for hist in (h_mt, h_ph):
        tot = sum(hist.values())
        f = np.array([hist.get(j, 0) for j in top]) / tot
        pe = p[np.argsort(-p)[:20]]
        assert np.all(np.abs(f - pe) < 6 * np.sqrt(pe / tot) + 2e-3)
