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
    assert size == 3 * 4 * nparam + 40 + len(ck._string_scalar_bytes(og)[0])
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
    assert os.path.getsize(os.path.join(vdir, 'variables.data-00000-of-00002')) == len(ck._string_scalar_bytes(og)[0])
    V2, d2, P2, M2, _, step = ck.load_variables(dest)
    assert (V2, d2, step) == (V, d, 100)


def _crc32c_py(data, crc=0):
    """Bitwise CRC-32C (Castagnoli, reflected 0x82F63B78): independent of the library's table."""
    crc ^= 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def test_string_entry_bytes_follow_tf_write_string_tensor():
    """A scalar DT_STRING entry laid out by the spec of TF's WriteStringTensor (tensor_bundle.cc):
    varint64 length, masked crc32c of the length as uint32 LE, the bytes; the entry crc32c runs over
    the uint32 length, the 4 checksum bytes and the string (not over the varint)."""
    import struct
    assert _crc32c_py(b'123456789') == 0xE3069283          # the CRC-32C check value
    s = b'x' * 200                                          # a 2-byte varint length
    raw, crc = ck._string_scalar_bytes(s)
    c = _crc32c_py(struct.pack('<I', 200))
    ck_bytes = struct.pack('<I', ck._mask(c))
    assert raw == bytes([0xC8, 0x01]) + ck_bytes + s
    assert crc == _crc32c_py(s, _crc32c_py(ck_bytes, c))


def test_index_layout_against_reference_pointer_sizes(tmp_path):
    """variables.index as TF's table builder writes it (prefix-compressed keys, restart interval
    16, shortest-successor index key; tensors in object-graph order, the object graph last).  The
    reference's pointers pin the 2-shard minus 1-shard index size of one model: 5,657 B
    (cc_rec_1000_regularization/variables/variables.index:3) - 5,501 B (recommender/variables/
    variables.index:3) = 156 B (81 shard-1 entries x 2 B of shard_id - the object graph's 6-B offset
    field).  The absolute size depends on the exact key set (TF absent: which metrics' accumulators
    hold the 4 scalar floats is unpinned), so it is checked within 5 % of 5,657."""
    V, d = 20884, 512
    lay = Layout(V, d)
    P = {n: np.zeros(lay.entries[n][1], np.float32) for n in NAMES}
    sizes = {}
    for shards in (1, 2):
        dest = str(tmp_path / f's{shards}')
        ck.save_model(dest, V, d, P, P, P, step=100, shards=shards)
        sizes[shards] = os.path.getsize(os.path.join(dest, 'variables', 'variables.index'))
        t = ck.read_bundle(os.path.join(dest, 'variables', 'variables'))   # crc-verified
        assert len(t) == 82
    assert sizes[2] - sizes[1] == 5657 - 5501
    assert abs(sizes[2] - 5657) < 0.05 * 5657, sizes


def test_saved_model_proto_mirrors_object_graph(tmp_path):
    """saved_model.pb (N2): a SavedModel proto whose SavedObjectGraph has the checkpoint object
    graph's nodes in the same order with the same children and slot variables; every variable node
    carries its bundle tensor's dtype / shape; the Dense layers carry model.py's configs (units,
    activation, fan-in) and the root the compile() training config (train.py:82-88)."""
    from cubecobrarecommender_amd.savedmodel import parse_saved_model
    V, d = 300, 64
    P = model_ref.init_params(V, d, seed=3, bias_std=0.01)
    M = {k: v * 0.5 for k, v in P.items()}
    dest = str(tmp_path / 'ml_files' / 'neg')
    ck.save_model(dest, V, d, P, M, M, step=4, reg=0.1, shards=2)
    sm = parse_saved_model(open(os.path.join(dest, 'saved_model.pb'), 'rb').read())
    assert sm['schema_version'] == 1 and sm['tags'] == ['serve']
    t = ck.read_bundle(os.path.join(dest, 'variables', 'variables'))
    og = ck.parse_object_graph(t[ck.OBJECT_GRAPH_KEY])
    assert len(sm['nodes']) == len(og)
    nvar = 0
    for a, b in zip(sm['nodes'], og):
        assert a['children'] == b['children'] and a['slots'] == b['slots']
        if b['attrs']:
            nvar += 1
            _, full, key = b['attrs'][0]
            assert a['kind'] == 'variable' and a['name'] == full
            assert a['shape'] == list(t[key].shape)
            assert a['dtype'] == (ck.DT_INT64 if t[key].dtype == np.int64 else ck.DT_FLOAT)
        else:
            assert a['kind'] == 'user_object'
    assert nvar == len(t) - 1                       # every bundle tensor but the graph string
    root = sm['nodes'][0]
    assert root['identifier'] == '_tf_keras_model' and root['metadata']['class_name'] == 'CC_Recommender'
    tc = root['metadata']['training_config']
    assert tc['loss'] == ['binary_crossentropy', 'kullback_leibler_divergence'] and tc['loss_weights'] == [1.0, 0.1]
    dense = {n['metadata']['name']: n['metadata']['config'] for n in sm['nodes']
             if n['kind'] == 'user_object' and n['identifier'] == '_tf_keras_layer'}
    assert len(dense) == 12
    assert (dense['encoder_e1']['units'], dense['encoder_e1']['activation']) == (d, 'relu')
    assert (dense['main_reconstruction']['units'], dense['main_reconstruction']['activation']) == (V, 'sigmoid')
    assert (dense['reg_reconstruction']['units'], dense['reg_reconstruction']['activation']) == (V, 'softmax')
    assert dense['encoder_bottleneck']['units'] == 64 and dense['main_d2']['units'] == 256
    trainable = [n for n in sm['nodes'] if n['kind'] == 'variable' and n['trainable']]
    assert len(trainable) == 24                      # the 12 kernels + 12 biases
    # the loader side still reads the directory
    V2, d2, P2, _, _, step = ck.load_variables(dest)
    assert (V2, d2, step) == (V, d, 4)
