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
    # data shard = weights + m + v (fp32) + 40 B of scalars + the object-graph string
    size = os.path.getsize(os.path.join(dest, 'variables', 'variables.data-00000-of-00001'))
    nparam = sum(int(np.prod(P[n].shape)) for n in NAMES)
    og = ck.read_bundle(os.path.join(dest, 'variables', 'variables'))[ck.OBJECT_GRAPH_KEY]
    assert size == 3 * 4 * nparam + 40 + len(ck._string_scalar_bytes(og))
    _, _, flat = ck.flat_params(dest)
    assert np.array_equal(Layout(V, d).unpack(flat)['decoder/reconstruct/kernel'], P['decoder/reconstruct/kernel'])


def test_object_graph_names_every_variable(tmp_path):
    """The _CHECKPOINTABLE_OBJECT_GRAPH entry: every saved tensor is an attribute of exactly one
    node, slot variables hang off the optimizer node with their original variable's node id, and
    the model's children follow model.py's attribute names."""
    V, d = 200, 64
    P = model_ref.init_params(V, d, seed=1)
    dest = str(tmp_path / 'm')
    ck.save_model(dest, V, d, P, P, P, step=3, metrics={'loss': (1.5, 3.0)})
    t = ck.read_bundle(os.path.join(dest, 'variables', 'variables'))
    nodes = ck.parse_object_graph(t[ck.OBJECT_GRAPH_KEY])
    keys = [k for nd in nodes for _, _, k in nd['attrs']]
    assert sorted(keys) == sorted(k for k in t if k != ck.OBJECT_GRAPH_KEY)
    assert [l for _, l in nodes[0]['children']] == ['encoder', 'decoder', 'decoder_for_reg', 'optimizer', 'keras_api']
    opt = nodes[[c for c, l in nodes[0]['children'] if l == 'optimizer'][0]]
    assert len(opt['slots']) == 2 * len(NAMES)
    for orig, slot, sv in opt['slots']:
        (_, _, okey), = nodes[orig]['attrs']
        (_, _, skey), = nodes[sv]['attrs']
        assert skey == okey.replace(ck.VAR_SUFFIX, f'/.OPTIMIZER_SLOT/optimizer/{slot}' + ck.VAR_SUFFIX)
    full = {k: f for nd in nodes for _, f, k in nd['attrs']}
    assert full['decoder/reconstruct/kernel' + ck.VAR_SUFFIX] == 'cc__recommender/decoder/main_reconstruction/kernel'
    assert t['keras_api/metrics/0/total' + ck.VAR_SUFFIX] == np.float32(1.5)
    assert t['keras_api/metrics/1/count' + ck.VAR_SUFFIX] == np.float32(0.0)


def test_two_shard_layout_matches_reference_pointer_sizes(tmp_path):
    """The reference's own Git-LFS pointers are the only known answers for ml_files/: at the
    reference checkpoint's |V| = 20,884, d = 512 every 2-shard save holds 391,661,320 B in its
    variables shard (ml_files/cc_rec_1000_regularization/variables/variables.data-00001-of-00002:3,
    and the same size in high_noise/ and high_req/) — weights + Adam m + v + 40 B of scalars — and
    the object graph alone in shard 0.  The writer's 2-shard save must give the same byte count."""
    V, d = 20884, 512
    lay = Layout(V, d)
    shapes = lay.entries
    P = {n: np.zeros(shapes[n][1], np.float32) for n in NAMES}
    assert sum(int(np.prod(a.shape)) for a in P.values()) == 32638440     # 1538 * V + 518,848
    dest = str(tmp_path / 'cc_rec')
    ck.save_model(dest, V, d, P, P, P, step=100, shards=2)
    vdir = os.path.join(dest, 'variables')
    assert os.path.getsize(os.path.join(vdir, 'variables.data-00001-of-00002')) == 391661320
    og = ck.read_bundle(os.path.join(vdir, 'variables'), verify=False)[ck.OBJECT_GRAPH_KEY]
    assert os.path.getsize(os.path.join(vdir, 'variables.data-00000-of-00002')) == len(ck._string_scalar_bytes(og))
    V2, d2, P2, M2, _, step = ck.load_variables(dest)
    assert (V2, d2, step) == (V, d, 100)
