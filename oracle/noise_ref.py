"""Noise function F and regulariser-row sampling — ORACLE (test infrastructure only).

Reference: ``src/ml/generator.py``
  * ``__init__`` :6-30  — ``neg_sampler = adj_mtx.sum(0) / adj_mtx.sum()`` (:30)
  * ``__getitem__`` :38-61 — B reg rows drawn iid with replacement ∝ neg_sampler (:47-51)
  * ``reset_indices`` :63-66 — per-epoch permutation
  * ``generate_data`` :74-103 — per cube: noise = clip(N(noise, std), .05, .8) (:86-90),
    k = int(n*noise) (:91), cut = k draws w/ replacement from includes (:92),
    add = k draws w/ replacement from excludes ∝ neg_sampler renormalised (:93-94),
    ycut = k//4 draws w/ replacement from the cut multiset (:95);
    x = cube - cut + add, y = cube - ycut (:96-101).

Two restatements of the same law:

``MTNoise``            replays the reference's own numpy legacy-MT19937 call sequence, so
                       with the same seed it reproduces the reference generator's batches
                       bit-for-bit (pinned by ``tests/golden/generator_*.npz``).
``philox_noise_batch`` the counter-based law the HIP kernel ``cc_noise_fwd`` implements:
                       every draw is a pure function of (seed, step, slot, kind, index, try)
                       through Philox4x32-10.  The add draws use rejection against the
                       global CDF of neg_sampler, which is exactly the renormalised law of
                       generator.py:93-94.  Bit-exact vs the GPU.
"""
import numpy as np

from .philox import philox4x32, u53, u53_open0, mulhi32
from .detmath import det_normal

KIND_NOISE, KIND_CUT, KIND_YCUT, KIND_ADD, KIND_ADD_FB, KIND_REG = 0, 1, 2, 3, 4, 5
ADD_MAX_TRIES = 256


def neg_sampler_of(y_mtx):
    """generator.py:30 — column mass of M~ normalised to a distribution (float64)."""
    y = np.asarray(y_mtx, dtype=np.float64)
    return y.sum(0) / y.sum()


def cdf_of(neg_sampler):
    """The normalised CDF numpy's ``choice(p=...)`` searches (float64, last entry 1.0)."""
    cdf = np.cumsum(np.asarray(neg_sampler, np.float64))
    cdf /= cdf[-1]
    return cdf


# ----------------------------------------------------------------------------------------
# MT19937 replay of the reference generator (bit-exact vs generator.py under np.random.seed)
# ----------------------------------------------------------------------------------------
class MTNoise:
    """Replays ``DataGenerator`` draws with a ``numpy.random.RandomState`` in the exact call
    order of generator.py:47-51 and :82-98.  Operates on sorted index lists instead of the
    dense f64 cube matrix; outputs are index lists (x, y) plus reg indices."""

    def __init__(self, rs, neg_sampler, num_cards, noise=0.2, noise_std=0.1):
        self.rs = rs
        self.ns = np.asarray(neg_sampler, np.float64)
        self.V = int(num_cards)
        self.noise = noise
        self.noise_std = noise_std

    def reg_indices(self, count):
        # generator.py:47-51
        return self.rs.choice(np.arange(self.V), count, p=self.ns)

    def cube(self, includes):
        """generator.py:83-98 for one cube; returns (x_list, y_list) as sorted int arrays."""
        includes = np.asarray(includes, np.int64)
        mask = np.zeros(self.V, bool)
        mask[includes] = True
        excludes = np.nonzero(~mask)[0]
        size = len(includes)
        noise = np.clip(self.rs.normal(self.noise, self.noise_std), a_min=0.05, a_max=0.8)
        k = int(size * noise)
        flip_include = self.rs.choice(includes, k)
        ns = self.ns[excludes] / self.ns[excludes].sum()
        flip_exclude = self.rs.choice(excludes, k, p=ns)
        y_flip_include = self.rs.choice(flip_include, k // 4)
        x = mask.copy()
        x[flip_include] = False
        x[flip_exclude] = True
        y = mask.copy()
        y[y_flip_include] = False
        return np.nonzero(x)[0], np.nonzero(y)[0]

    def batch(self, cube_lists):
        """generator.py:44-56: reg draws first, then the per-cube loop."""
        reg = self.reg_indices(len(cube_lists))
        xs, ys = [], []
        for inc in cube_lists:
            x, y = self.cube(inc)
            xs.append(x)
            ys.append(y)
        return xs, ys, reg


# ----------------------------------------------------------------------------------------
# Counter-based (Philox) restatement — the law of the HIP kernel cc_noise_fwd
# ----------------------------------------------------------------------------------------
def _rng(seed, step, slot, kind, idx, tries=0):
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32((seed >> 32) & 0xFFFFFFFF)
    c1 = (np.uint32(kind) << np.uint32(24)) | np.asarray(tries, np.uint32)
    return philox4x32(idx, c1, np.uint32(slot), np.uint32(step & 0xFFFFFFFF), k0, k1)


def philox_noise_level(seed, step, slot, mean, std):
    o0, o1, o2, o3 = _rng(seed, step, slot, KIND_NOISE, np.uint32(0))
    u1 = u53_open0(o0, o1)
    u2 = u53(o2, o3)
    z = det_normal(u1, u2)
    lvl = float(mean) + float(std) * float(z)
    return min(max(lvl, 0.05), 0.8)


def _searchsorted_right(cdf, u):
    return np.searchsorted(cdf, u, side='right')


def philox_cube(includes, cdf, neg_sampler, seed, step, slot, mean=0.2, std=0.1):
    """One cube of F under the counter-based law.  Returns (x_sorted, y_sorted, k)."""
    inc = np.asarray(includes, np.int64)
    n = len(inc)
    V = len(cdf)
    lvl = philox_noise_level(seed, step, slot, mean, std)
    k = int(float(n) * lvl)
    in_cube = np.zeros(V, bool)
    in_cube[inc] = True
    cut_cards = np.zeros(0, np.int64)
    ycut_cards = np.zeros(0, np.int64)
    add_cards = np.zeros(0, np.int64)
    if k > 0:
        i = np.arange(k, dtype=np.uint32)
        o0 = _rng(seed, step, slot, KIND_CUT, i)[0]
        pos = mulhi32(o0, n)
        cut_cards = inc[pos]
        nq = k // 4
        if nq > 0:
            q = mulhi32(_rng(seed, step, slot, KIND_YCUT, np.arange(nq, dtype=np.uint32))[0], k)
            ycut_cards = cut_cards[q]
        # add draws: rejection against the global CDF, up to ADD_MAX_TRIES tries per draw
        adds = np.full(k, -1, np.int64)
        pending = np.arange(k)
        for t in range(ADD_MAX_TRIES):
            if len(pending) == 0:
                break
            a0, a1, _, _ = _rng(seed, step, slot, KIND_ADD, pending.astype(np.uint32), t)
            j = _searchsorted_right(cdf, u53(a0, a1))
            ok = ~in_cube[j]
            adds[pending[ok]] = j[ok]
            pending = pending[~ok]
        if len(pending):
            ns = np.asarray(neg_sampler, np.float64)
            ex = np.nonzero(~in_cube)[0]
            s = 0.0
            for jj in ex:  # sequential fp64 sum, ascending card id
                s += ns[jj]
            for i_draw in pending:
                if s <= 0.0:
                    continue
                f0, f1, _, _ = _rng(seed, step, slot, KIND_ADD_FB, np.uint32(i_draw))
                u = float(u53(f0, f1)) * s
                acc = 0.0
                pick = -1
                last_pos = -1
                for jj in ex:
                    if ns[jj] > 0.0:
                        last_pos = jj
                    acc += ns[jj]
                    if acc > u:
                        pick = jj
                        break
                if pick < 0:
                    pick = last_pos
                adds[i_draw] = pick
        add_cards = adds[adds >= 0]
    x = in_cube.copy()
    x[cut_cards] = False
    x[add_cards] = True
    y = in_cube.copy()
    y[ycut_cards] = False
    return np.nonzero(x)[0], np.nonzero(y)[0], k


def philox_reg_indices(cdf, seed, step, slot_base, count):
    """generator.py:47-51 (B reg rows iid ∝ neg_sampler) on Philox: slot s draws
    searchsorted_right(cdf, u53(Philox(seed; 0, REG<<24, s, step)))."""
    slots = np.uint32(slot_base) + np.arange(count, dtype=np.uint32)
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32((seed >> 32) & 0xFFFFFFFF)
    o0, o1, _, _ = philox4x32(np.uint32(0), np.uint32(KIND_REG << 24), slots,
                              np.uint32(step & 0xFFFFFFFF), k0, k1)
    u = u53(o0, o1)
    return _searchsorted_right(cdf, u).astype(np.int64)


def owner_reg_rows(cdf, seed, step, slots, lo, hi, cap):
    """SURVEY §8(e) owner computes (csrc/noise.hip cc_reg_rows): the step's `slots` global reg draws
    (slot s exactly as a one-process run of batch `slots` draws it), the cards in [lo, hi) kept in
    slot order, padded with -1 to `cap`.  Returns (reg_idx [cap], owned count, overflow flag)."""
    j = philox_reg_indices(cdf, seed, step, 0, slots)
    own = j[(j >= lo) & (j < hi)]
    out = np.full(cap, -1, np.int64)
    n = min(len(own), cap)
    out[:n] = own[:n]
    return out, len(own), len(own) > cap


def philox_noise_batch(cube_lists, cdf, neg_sampler, seed, step, slot_base=0,
                       mean=0.2, std=0.1, with_reg=True):
    xs, ys, ks = [], [], []
    for b, inc in enumerate(cube_lists):
        x, y, k = philox_cube(inc, cdf, neg_sampler, seed, step, slot_base + b, mean, std)
        xs.append(x)
        ys.append(y)
        ks.append(k)
    reg = philox_reg_indices(cdf, seed, step, slot_base, len(cube_lists)) if with_reg else None
    return xs, ys, reg, np.array(ks)
