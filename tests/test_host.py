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
    """SURVEY §8(e) owner computes: M~ row shards at equal cumulative neg_sampler mass; the ranks'
    owned rows of the global draws partition exactly the one-process draws (slot order kept), and
    the static capacity covers the Binomial(world*B, m_r) owned count at 6 sigma."""
    import pytest
    from cubecobrarecommender_amd.trainer import full_rows, owner_capacity, reg_row_shards
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
    B, W = 512, 8
    b, m = reg_row_shards(cdf, W)
    cap = owner_capacity(m, B, W)
    assert cap % 32 == 0 and W * B * m.max() < cap <= W * B
    flat = np.full(8, 1 / 8)        # the bench's shards sit within 0.1 % of equal mass
    assert owner_capacity(flat, 512, 8) == 640 and owner_capacity(flat[:2] * 4, 512, 2) == 640
    worst = 0
    for step in range(40):
        one = noise_ref.philox_reg_indices(cdf, 11, step, 0, W * B)      # one process, batch W*B
        parts = []
        for r in range(W):
            rows, n, over = noise_ref.owner_reg_rows(cdf, 11, step, W * B, int(b[r]), int(b[r + 1]), cap)
            assert not over and np.all(rows[n:] == -1)
            assert np.all((rows[:n] >= b[r]) & (rows[:n] < b[r + 1]))
            parts.append(rows[:n])
            worst = max(worst, n)
        # every draw is owned by exactly one rank, in slot order within the rank
        merged = np.concatenate(parts)
        assert np.array_equal(np.sort(merged), np.sort(one))
        for r in range(W):
            sel = one[(one >= b[r]) & (one < b[r + 1])]
            assert np.array_equal(parts[r], sel)
    assert worst <= cap
    lo_hi = [full_rows(22000, 8, r) for r in range(8)]
    assert lo_hi[0][0] == 0 and lo_hi[-1][1] == 22000
    assert all(lo_hi[i][1] == lo_hi[i + 1][0] for i in range(7))
    heavy = np.full(10, 0.01)
    heavy[0] = 0.91
    with pytest.raises(ValueError):
        reg_row_shards(np.cumsum(heavy) / heavy.sum(), 4)


def test_fused_kernel_extent_gates():
    """The fused D2 kernel and the split-K dX take 32-bit buffer extents: above them the trainer
    must pick the unfused paths instead of failing at the first step."""
    from cubecobrarecommender_amd.trainer import dx_splitk_fits, fused_reg_fits
    assert fused_reg_fits(22000, 22000, 512)
    assert fused_reg_fits(23170, 23170, 512)
    assert not fused_reg_fits(23171, 23171, 512)       # hi * V * 4 > 2^31 - 1
    assert fused_reg_fits(23171 // 2, 23171, 512)       # a row shard ending below the limit
    assert dx_splitk_fits(512, 22000, 256)
    assert not dx_splitk_fits(33000, 33000, 256)       # full-mode dZ (Breg ~ V) past 2 GB


def test_names_unidecode_restatement():
    """N3 (ml_recommend.py:44): unidecode(name.lower()) restated for Latin-1 / Latin Extended-A,
    Greek, Cyrillic, punctuation and number forms, Hangul and kana (Unidecode 1.1.1's tables);
    ASCII passes through unchanged, combining marks vanish, private use maps to ''."""
    from cubecobrarecommender_amd.names import normalize, unidecode
    cases = {
        'Lim-Dûl the Necromancer': 'lim-dul the necromancer', 'Æther Vial': 'aether vial',
        'Jötun Grunt': 'jotun grunt', 'Déjà Vu': 'deja vu', 'Ifh-Bíff Efreet': 'ifh-biff efreet',
        'Juzám Djinn': 'juzam djinn', 'Dandân': 'dandan', 'Sol Ring': 'sol ring',
        'Phyrexian™ — “Obliterator”…': 'phyrexian(tm) -- "obliterator"...',
        'Łukasz ½ × ÷': 'lukasz  1/2 x /', 'Ŀ Đ ħ ı ĸ ŉ Ŋ ŧ ſ ß þ': "l d h i q 'n ng t s ss th",
        'Ελλάδα': 'ellada', 'Москва': 'moskva', 'Ⅻ': 'xii', 'Hồ Chí Minh': 'ho chi minh',
        'µ°¿¡': 'udeg?!', 'á': 'a', '\U000F0000x': 'x',
    }
    for raw, want in cases.items():
        assert normalize(raw) == want, (raw, normalize(raw), want)
    assert unidecode('ÆON') == 'AEON' and unidecode('plain ascii') == 'plain ascii'
    # every restated Latin-1 / Extended-A entry is ASCII
    for cp in range(0x80, 0x180):
        assert unidecode(chr(cp)).isascii(), hex(cp)
    # Korean printings: Hangul syllables as initial + medial + final jamo romanisation (unidecode's
    # xac..xd7 tables); Japanese kana (x030, Kunrei style).  Parity unpinned (no reference output)
    assert unidecode('안녕') == 'annyeong' and unidecode('한국어') == 'hangugeo'
    assert unidecode('힣') == 'hih' and unidecode('가') == 'ga'
    assert unidecode('ドラゴン') == 'doragon' and unidecode('しつ') == 'situ' and unidecode('カード') == 'ka-do'
    for cp in list(range(0xAC00, 0xD7A4, 97)) + list(range(0x3041, 0x3095)) + list(range(0x30A1, 0x30F5)):
        assert unidecode(chr(cp)).isascii() and unidecode(chr(cp)), hex(cp)


def test_dp_layout_w1_chunks_any_world():
    """W1 row chunks stay whole bucket shards for worlds that are not powers of two (ADVICE r05:
    d = 1024 with world 3 / 6 used to trip the alignment assert at Trainer construction)."""
    from cubecobrarecommender_amd.layout import Layout
    for world in (1, 2, 3, 5, 6, 7, 8):
        for d, chunks in ((256, 1), (1024, 2), (1024, 3), (512, 4)):
            lay = Layout(22000, d, align=64 * world, group_biases=True, w1_chunks=chunks)
            for name, lo, hi in lay.buckets(True):
                assert (hi - lo) % (64 * world) == 0, (world, d, name)
            assert all(r0 % 64 == 0 for r0, _ in lay.w1_chunks)
            assert lay.w1_chunks[0][0] == 0 and lay.w1_chunks[-1][1] == 22000


def test_bench_rank_argv_passes_torchrun_parser(monkeypatch):
    """bench.py --gpus N starts its ranks through torch.distributed.run, whose parser rejects an
    ambiguous abbreviation of its own options before the script's arguments: `--d` is renamed."""
    import sys

    import pytest
    from torch.distributed.run import get_args_parser

    import bench
    argv = ['--gpus', '4', '--d', '1024', '--dtype', 'fp8', '--reg', '0.1', '--d=512']
    out = bench.child_argv(argv)
    assert out == ['--gpus', '4', '--dim', '1024', '--dtype', 'fp8', '--reg', '0.1', '--dim=512']
    ns = get_args_parser().parse_args(['--nnodes=1', '--nproc-per-node=4', 'bench.py', *out])
    assert ns.training_script_args == out
    with pytest.raises(SystemExit):       # the unrenamed form is what failed
        get_args_parser().parse_args(['--nnodes=1', 'bench.py', *argv])
    monkeypatch.setattr(sys, 'argv', ['bench.py', *out])
    assert bench.parse().d == 512
