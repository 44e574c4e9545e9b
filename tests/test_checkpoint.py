"""CPU tests: ml_files/<name>/ tensor-bundle checkpoints (write -> read round trip, format checks)."""
import os
import struct

import numpy as np

from cubecobrarecommender_amd import checkpoint as ck
from cubecobrarecommender_amd.layout import NAMES, Layout
from oracle import model_ref


def test_bundle_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    t = {'a/b' + ck.VAR_SUFFIX: rng.standard_normal((3, 5)).astype(np.float32),
         'optimizer/iter' + ck.VAR_SUFFIX: np.array(7, np.int64),
         'z' + ck.VAR_SUFFIX: np.zeros(0, np.float32)}
    pre = str(tmp_path / 'variables' / 'variables')
    ck.write_bundle(pre, t)
    got = ck.read_bundle(pre)
    for k in t:
        assert np.array_equal(got[k], t[k]) and got[k].dtype == t[k].dtype
    # format: SSTable magic, masked crc32c on the entries
    idx = open(pre + '.index', 'rb').read()
    assert struct.unpack('<Q', idx[-8:])[0] == ck.MAGIC
    assert ck.crc32c(b'123456789') == 0xe3069283
    assert ck._unmask(ck._mask(0x12345678)) == 0x12345678


def test_model_save_load(tmp_path):
    V, d = 300, 64
    P = model_ref.init_params(V, d, seed=3, bias_std=0.01)
    M = {k: v * 0.5 for k, v in P.items()}
    dest = str(tmp_path / 'ml_files' / 'recommender')
    ck.save_model(dest, V, d, P, M, M, step=12)
    assert os.path.exists(os.path.join(dest, 'saved_model.pb'))
    assert os.path.exists(os.path.join(dest, 'variables', 'variables.data-00000-of-00001'))
    V2, d2, P2, M2, V2s, step = ck.load_variables(dest)
    assert (V2, d2, step) == (V, d, 12)
    for n in NAMES:
        assert np.array_equal(P2[n], P[n]) and np.array_equal(M2[n], M[n])
    # data shard = weights + m + v (fp32) + optimizer scalars, as the reference checkpoint sizes imply
    size = os.path.getsize(os.path.join(dest, 'variables', 'variables.data-00000-of-00001'))
    nparam = sum(int(np.prod(P[n].shape)) for n in NAMES)
    assert size == 3 * 4 * nparam + 8 + 4 * 4
    _, _, flat = ck.flat_params(dest)
    assert np.array_equal(Layout(V, d).unpack(flat)['decoder/reconstruct/kernel'], P['decoder/reconstruct/kernel'])
