"""``ml_files/<name>/`` checkpoint layout — TF tensor-bundle reader/writer.

Reference: ``autoencoder.save(dest, save_format='tf')`` (src/ml/train.py:112-115) writes a Keras
SavedModel directory ``ml_files/<name>/{saved_model.pb, variables/variables.index,
variables/variables.data-0000K-of-0000N}``; the recommenders load it with
``keras.models.load_model`` (src/scripts/ml_recommend.py:54, web/ml_recommend_web.py:37).

The variables are a TF *tensor bundle*:
  * ``variables.data-*``: raw little-endian tensor bytes;
  * ``variables.index``: a LevelDB-format SSTable.  Key ``""`` -> BundleHeaderProto
    {num_shards, endianness, version}; key ``<object path>/.ATTRIBUTES/VARIABLE_VALUE`` ->
    BundleEntryProto {dtype, shape, shard_id, offset, size, crc32c (masked)}.
Object paths follow the attribute names of model.py (``encoder/encoded_1/kernel`` ...), Adam slots
``<var>/.OPTIMIZER_SLOT/optimizer/{m,v}/...`` and ``optimizer/iter`` etc.

The writer produces a bundle any tensor-bundle reader (tf.train.load_checkpoint) can parse, with
the TF2 `_CHECKPOINTABLE_OBJECT_GRAPH` string (a TrackableObjectGraph proto naming every saved
variable, its Keras layer name and Adam slots); the reader parses such files (multi-block,
prefix-compressed, multi-shard, string tensors).  The reference's Git-LFS pointers pin the data
sizes (12 * P + 40 B of variables at |V| = 20,884, d = 512; tests/test_checkpoint.py checks the
writer against them); the byte contents of files written by TF itself stay unpinned (no real
checkpoint exists in this pipeline).  ``saved_model.pb`` is a SavedModel proto whose
SavedObjectGraph mirrors the object graph node for node (savedmodel.py; the traced functions, which
only TF can produce, are absent), and ``ccrec_config.json`` records (V, d).
"""
import json
import os
import struct

import numpy as np

from . import _lib as L
from .layout import NAMES, Layout

MAGIC = 0xdb4775248b80fb57
DT_FLOAT, DT_STRING, DT_INT64 = 1, 7, 9
_NP = {DT_FLOAT: np.float32, DT_INT64: np.int64}
VAR_SUFFIX = '/.ATTRIBUTES/VARIABLE_VALUE'
OBJECT_GRAPH_KEY = '_CHECKPOINTABLE_OBJECT_GRAPH'

# Keras layer names of model.py (Dense(..., name=...)): the variables' TF names (full_name in the
# object graph), e.g. encoder/encoded_1 -> 'encoder_e1' (model.py:27), decoder/reconstruct ->
# 'main_reconstruction' (model.py:64, Decoder("main", ...) at :94)
_LAYER_NAMES = {'encoder/encoded_1': 'encoder_e1', 'encoder/encoded_2': 'encoder_e2',
                'encoder/encoded_3': 'encoder_e3', 'encoder/bottleneck': 'encoder_bottleneck'}
for _pre, _tag in (('decoder', 'main'), ('decoder_for_reg', 'reg')):
    _LAYER_NAMES.update({f'{_pre}/decoded_1': f'{_tag}_d1', f'{_pre}/decoded_2': f'{_tag}_d2',
                         f'{_pre}/decoded_3': f'{_tag}_d3', f'{_pre}/reconstruct': f'{_tag}_reconstruction'})
# Adam's scalar variables (Keras OptimizerV2: `iter` int64 + the float hyper-parameters) and the
# compiled metrics' accumulators (keras_api/metrics/<i>/{total,count}).  The reference's own
# checkpoints pin their total: the GPU shard of every 2-shard save is 391,661,320 B = 12 * P + 40
# at |V| = 20,884, d = 512 (P = 32,638,440: weights + Adam m + v), i.e. 40 B of scalars beside the
# object graph (shard 0, 18,317 B).  The pointer sizes also pin the NUMBER of shard-1 entries: the
# index of the 2-shard save (5,657 B) is 156 B larger than the same model's 1-shard save
# (ml_files/recommender, 5,501 B), = 2 B of shard_id per shard-1 entry minus the 6-B offset field
# of the object graph written last in the 1-shard file -> 81 entries = 72 weight / m / v tensors +
# 9 scalars, i.e. iter (8 B) + 8 float32 = 40 B: the 4 optimizer hypers and 4 metric floats.
# WHICH metric accumulators those 4 floats are is an inference (unpinned: TF is absent): two
# Mean metrics, taken here as 'loss' and the first output's loss.
OPT_HYPERS = ('learning_rate', 'beta_1', 'beta_2', 'decay')
METRICS = ('loss', 'output_1_loss')


def crc32c(data, crc=0):
    buf = memoryview(data).cast('B')
    arr = np.frombuffer(buf, np.uint8)
    return L.lib().cc_crc32c(crc, arr.ctypes.data, arr.size)


def _mask(c):
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xa282ead8) & 0xFFFFFFFF


def _unmask(c):
    r = (c - 0xa282ead8) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------------------- protobuf bits
def _varint(v):
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(b, i):
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def _field(num, wire, payload):
    key = _varint((num << 3) | wire)
    if wire == 0:
        return key + _varint(payload)
    if wire == 2:
        return key + _varint(len(payload)) + payload
    if wire == 5:
        return key + struct.pack('<I', payload)
    raise ValueError(wire)


def _parse(b):
    """Minimal protobuf parse -> {field: [values]} (varint / len / fixed32 / fixed64)."""
    out, i = {}, 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, i = _read_varint(b, i)
        elif wire == 2:
            n, i = _read_varint(b, i)
            v = bytes(b[i:i + n])
            i += n
        elif wire == 5:
            v = struct.unpack_from('<I', b, i)[0]
            i += 4
        elif wire == 1:
            v = struct.unpack_from('<Q', b, i)[0]
            i += 8
        else:
            raise ValueError(f'wire type {wire}')
        out.setdefault(num, []).append(v)
    return out


def _header_proto(num_shards):
    return _field(1, 0, num_shards) + _field(3, 2, _field(1, 0, 1))   # version {producer: 1}


def _entry_proto(dtype, shape, shard, offset, size, crc):
    shp = b''.join(_field(2, 2, _field(1, 0, int(d))) for d in shape)
    out = _field(1, 0, dtype) + _field(2, 2, shp)
    if shard:
        out += _field(3, 0, shard)
    if offset:
        out += _field(4, 0, offset)
    out += _field(5, 0, size) + _field(6, 5, crc)
    return out


# ---------------------------------------------------------------------------- SSTable
# TF's table builder (tensorflow/core/lib/io/table_builder.cc, the LevelDB format): keys
# prefix-compressed against the previous key, a restart point every RESTART_INTERVAL entries
# (table::Options default 16; the index block restarts at every entry), blocks of ~BLOCK_SIZE bytes
# (default 256 KB), each followed by a 1-byte compression type (0: none) and a masked crc32c.
RESTART_INTERVAL = 16
BLOCK_SIZE = 262144


def _block(entries, interval=RESTART_INTERVAL):
    out = bytearray()
    restarts = []
    last = b''
    for i, (k, v) in enumerate(entries):
        shared = 0
        if i % interval == 0:
            restarts.append(len(out))
        else:
            n = min(len(last), len(k))
            while shared < n and last[shared] == k[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack('<I', r)
    out += struct.pack('<I', len(restarts))
    return bytes(out)


def _short_successor(k):
    """BytewiseComparator::FindShortSuccessor: the shortest key >= k (first non-0xff byte + 1)."""
    for i, c in enumerate(k):
        if c != 0xFF:
            return k[:i] + bytes([c + 1])
    return k


def _short_separator(a, b):
    """BytewiseComparator::FindShortestSeparator: a short key in [a, b)."""
    n = min(len(a), len(b))
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    if i < n and a[i] < 0xFF and a[i] + 1 < b[i]:
        return a[:i] + bytes([a[i] + 1])
    return a


def _write_table(path, entries):
    entries = sorted(entries, key=lambda kv: kv[0])
    f = bytearray()

    def put_block(data):
        off = len(f)
        f.extend(data)
        f.append(0)                                   # no compression
        f.extend(struct.pack('<I', _mask(crc32c(data + b'\x00'))))
        return off, len(data)

    # data blocks of ~BLOCK_SIZE raw bytes; the index names each by a separator key
    index, blk, size = [], [], 0
    for j, (k, v) in enumerate(entries):
        blk.append((k, v))
        size += len(k) + len(v) + 8
        if size >= BLOCK_SIZE and j + 1 < len(entries):
            off, n = put_block(_block(blk))
            index.append((_short_separator(k, entries[j + 1][0]), _varint(off) + _varint(n)))
            blk, size = [], 0
    off, n = put_block(_block(blk))
    index.append((_short_successor(blk[-1][0]) if blk else b'', _varint(off) + _varint(n)))
    m_off, m_len = put_block(_block([]))
    i_off, i_len = put_block(_block(index, interval=1))
    footer = _varint(m_off) + _varint(m_len) + _varint(i_off) + _varint(i_len)
    footer += b'\x00' * (40 - len(footer)) + struct.pack('<Q', MAGIC)
    f.extend(footer)
    with open(path, 'wb') as fh:
        fh.write(bytes(f))


def _read_block(buf, off, size):
    data = buf[off:off + size]
    n = struct.unpack_from('<I', data, size - 4)[0]
    end = size - 4 - 4 * n
    out, i, last = [], 0, b''
    while i < end:
        shared, i = _read_varint(data, i)
        nsh, i = _read_varint(data, i)
        vlen, i = _read_varint(data, i)
        key = last[:shared] + bytes(data[i:i + nsh])
        i += nsh
        out.append((key, bytes(data[i:i + vlen])))
        i += vlen
        last = key
    return out


def _read_table(path):
    buf = open(path, 'rb').read()
    if struct.unpack_from('<Q', buf, len(buf) - 8)[0] != MAGIC:
        raise ValueError(f'{path}: not an SSTable')
    footer = buf[len(buf) - 48:]
    _, i = _read_varint(footer, 0)
    _, i = _read_varint(footer, i)
    i_off, i = _read_varint(footer, i)
    i_len, i = _read_varint(footer, i)
    out = []
    for _, handle in _read_block(buf, i_off, i_len):
        off, j = _read_varint(handle, 0)
        size, _ = _read_varint(handle, j)
        if buf[off + size] != 0:
            raise ValueError('compressed SSTable blocks are not supported')
        out.extend(_read_block(buf, off, size))
    return out


# ---------------------------------------------------------------------------- bundle
def _string_scalar_bytes(b):
    """A scalar DT_STRING tensor in a bundle data file (TF tensor_bundle.cc WriteStringTensor):
    the varint64 element length, the masked crc32c of the lengths taken as uint32 LE (uint64 above
    2^32 - 1), then the bytes.  Returns (raw bytes, entry crc): the entry's crc32c runs over the
    uint32 lengths, the 4 masked-checksum bytes and the string bytes (not over the varints)."""
    n = len(b)
    lens = struct.pack('<I', n) if n <= 0xFFFFFFFF else struct.pack('<Q', n)
    c = crc32c(lens)
    ck = struct.pack('<I', _mask(c))
    return _varint(n) + ck + b, crc32c(b, crc32c(ck, c))


def write_bundle(prefix, tensors, shard_of=None):
    """tensors: dict key -> numpy array (float32 / int64) or bytes (a scalar DT_STRING), in the
    order the data files receive them (TF writes the saveables in object-graph order, the object
    graph string last; the index is sorted by key).  Writes <prefix>.index +
    <prefix>.data-0000K-of-0000N; shard_of(key) -> shard id (default: one shard).  TF's
    multi-device saver writes one shard per device (the object graph on the CPU shard, the
    variables on the GPU shard), which the reference's 2-shard checkpoints show."""
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    shard_of = shard_of or (lambda key: 0)
    nshards = 1 + max((shard_of(k) for k in tensors), default=0)
    entries = [(b'', _header_proto(nshards))]
    files = [open(f'{prefix}.data-{s:05d}-of-{nshards:05d}', 'wb') for s in range(nshards)]
    offs = [0] * nshards
    try:
        for key in tensors:
            sh = shard_of(key)
            val = tensors[key]
            if isinstance(val, (bytes, bytearray)):
                dt, shape = DT_STRING, ()
                raw, crc = _string_scalar_bytes(bytes(val))
            else:
                a = np.array(val, order="C", copy=True)   # keeps 0-d scalars 0-d
                dt = DT_FLOAT if a.dtype == np.float32 else DT_INT64
                a = a.astype(_NP[dt], copy=False)
                shape, raw = a.shape, a.tobytes()
                crc = crc32c(raw)
            files[sh].write(raw)
            entries.append((key.encode(), _entry_proto(dt, shape, sh, offs[sh], len(raw), _mask(crc))))
            offs[sh] += len(raw)
    finally:
        for fh in files:
            fh.close()
    _write_table(prefix + '.index', entries)


def read_bundle(prefix, verify=True):
    """-> {key: numpy array (float32 / int64) or bytes (scalar DT_STRING)}."""
    ents = _read_table(prefix + '.index')
    header = _parse(dict(ents)[b''])
    nshards = header.get(1, [1])[0]
    shards = [np.memmap(f'{prefix}.data-{s:05d}-of-{nshards:05d}', np.uint8, 'r') for s in range(nshards)]
    out = {}
    for k, v in ents:
        if k == b'':
            continue
        e = _parse(v)
        dt = e.get(1, [0])[0]
        if dt not in _NP and dt != DT_STRING:
            continue
        shape = [(_parse(dim).get(1, [0])[0]) for dim in _parse(e[2][0]).get(2, [])] if 2 in e else []
        shard, off, size = e.get(3, [0])[0], e.get(4, [0])[0], e.get(5, [0])[0]
        raw = np.asarray(shards[shard][off:off + size])
        if dt == DT_STRING:   # TF's string layout (tensor_bundle.cc ReadStringTensor)
            if shape:
                raise ValueError(f'{k!r}: only scalar strings are supported')
            b = raw.tobytes()
            n, i = _read_varint(b, 0)
            lens = struct.pack('<I', n) if n <= 0xFFFFFFFF else struct.pack('<Q', n)
            c = crc32c(lens)
            if verify and _unmask(struct.unpack_from('<I', b, i)[0]) != c:
                raise ValueError(f'length crc mismatch for {k!r}')
            val = b[i + 4:i + 4 + n]
            if verify and 6 in e and _unmask(e[6][0]) != crc32c(val, crc32c(b[i:i + 4], c)):
                raise ValueError(f'crc mismatch for {k!r}')
            out[k.decode()] = val
            continue
        if verify and 6 in e and _unmask(e[6][0]) != crc32c(raw):
            raise ValueError(f'crc mismatch for {k!r}')
        out[k.decode()] = raw.view(_NP[dt]).reshape(shape).copy()
    return out


# ---------------------------------------------------------------------------- object graph
def object_graph(keys, metrics=METRICS):
    """TrackableObjectGraph proto (tensorflow/core/protobuf/trackable_object_graph.proto) of the
    model's checkpoint — the `_CHECKPOINTABLE_OBJECT_GRAPH` string a TF2 checkpoint carries:
    root (CC_Recommender, model.py:82-98) -> encoder / decoder / decoder_for_reg -> Dense layers
    -> kernel / bias; optimizer -> iter + hypers, with slot_variables (m, v) per model variable;
    keras_api -> metrics -> <i> -> total / count.  `keys`: the checkpoint keys written (so the
    graph names exactly the saved tensors).
      TrackableObject: children=1 {node_id=1, local_name=2}, attributes=2 {name=1, full_name=2,
      checkpoint_key=3}, slot_variables=3 {original_variable_node_id=1, slot_name=2,
      slot_variable_node_id=3}."""
    keys = set(keys)
    nodes = [{'children': [], 'attrs': [], 'slots': []}]

    def new(parent, local):
        nodes.append({'children': [], 'attrs': [], 'slots': []})
        nodes[parent]['children'].append((len(nodes) - 1, local))
        return len(nodes) - 1

    def var(node, path, full):
        nodes[node]['attrs'].append(('VARIABLE_VALUE', full, path + VAR_SUFFIX))

    var_node = {}
    subs = {}
    for n in NAMES:
        if n + VAR_SUFFIX not in keys:
            continue
        sub, layer, w = n.split('/')
        if sub not in subs:
            subs[sub] = (new(0, sub), {})
        sid, layers = subs[sub]
        if layer not in layers:
            layers[layer] = new(sid, layer)
        vid = new(layers[layer], w)
        var(vid, n, f'cc__recommender/{sub}/{_LAYER_NAMES[sub + "/" + layer]}/{w}')
        var_node[n] = vid
    if f'optimizer/iter{VAR_SUFFIX}' in keys:
        opt = new(0, 'optimizer')
        for h in ('iter',) + OPT_HYPERS:
            if f'optimizer/{h}{VAR_SUFFIX}' in keys:
                var(new(opt, h), f'optimizer/{h}', f'Adam/{h}')
        for n, vid in var_node.items():
            for slot in ('m', 'v'):
                path = f'{n}/.OPTIMIZER_SLOT/optimizer/{slot}'
                if path + VAR_SUFFIX in keys:
                    nodes.append({'children': [], 'attrs': [], 'slots': []})
                    sv = len(nodes) - 1
                    sub, layer, w = n.split('/')
                    var(sv, path, f'Adam/cc__recommender/{sub}/{_LAYER_NAMES[sub + "/" + layer]}/{w}/{slot}')
                    nodes[opt]['slots'].append((vid, slot, sv))
    if any(k.startswith('keras_api/metrics/') for k in keys):
        api = new(0, 'keras_api')
        ml = new(api, 'metrics')
        for i, name in enumerate(metrics):
            if f'keras_api/metrics/{i}/total{VAR_SUFFIX}' not in keys:
                continue
            mi = new(ml, str(i))
            for w in ('total', 'count'):
                var(new(mi, w), f'keras_api/metrics/{i}/{w}', f'{name}/{w}')
    out = b''
    for nd in nodes:
        body = b''.join(_field(1, 2, _field(1, 0, c) + _field(2, 2, l.encode())) for c, l in nd['children'])
        body += b''.join(_field(2, 2, _field(1, 2, a.encode()) + _field(2, 2, f.encode()) + _field(3, 2, k.encode()))
                         for a, f, k in nd['attrs'])
        body += b''.join(_field(3, 2, _field(1, 0, o) + _field(2, 2, sn.encode()) + _field(3, 0, sv))
                         for o, sn, sv in nd['slots'])
        out += _field(1, 2, body)
    return out


def parse_object_graph(b):
    """-> list of nodes {'children': [(node_id, local_name)], 'attrs': [(name, full_name, key)],
    'slots': [(orig_node, slot_name, slot_node)]} (the inverse of object_graph)."""
    nodes = []
    for body in _parse(b).get(1, []):
        f = _parse(body)
        ch = [(_parse(c).get(1, [0])[0], _parse(c).get(2, [b''])[0].decode()) for c in f.get(1, [])]
        at = [tuple(_parse(a).get(i, [b''])[0].decode() for i in (1, 2, 3)) for a in f.get(2, [])]
        sl = [(_parse(x).get(1, [0])[0], _parse(x).get(2, [b''])[0].decode(), _parse(x).get(3, [0])[0])
              for x in f.get(3, [])]
        nodes.append({'children': ch, 'attrs': at, 'slots': sl})
    return nodes


# ---------------------------------------------------------------------------- model files
def save_model(dest, V, d, params, m=None, v=None, step=0, lr=1e-3, beta1=0.9, beta2=0.999,
               metrics=None, shards=1, reg=0.0):
    """ml_files/<name>/ as train.py:112-115 lays it out.  params/m/v: dict name -> array.
    metrics: {'loss': (total, count), 'output_1_loss': (total, count)} — the compiled metrics'
    accumulators after fit (zeros when absent; written with the optimizer state).  shards=2: the
    object graph in shard 0 and every variable in shard 1, as the reference's GPU-trained
    checkpoints are laid out (ml_files/cc_rec_1000_regularization/variables/)."""
    os.makedirs(os.path.join(dest, 'variables'), exist_ok=True)
    # data-file order = TF's saveable order (the object graph's breadth-first node order,
    # util.py / graph_view.py): depth 2 the optimizer's own variables (iter, then the hypers in
    # sorted-name creation order), depth 3 the Dense kernels / biases, depth 4 the metrics'
    # accumulators, then the slot variables (all m, then all v: OptimizerV2 slot-name order), and
    # the object-graph string last
    t = {}
    if m is not None:
        t['optimizer/iter' + VAR_SUFFIX] = np.array(step, np.int64)
        for h, val in sorted(zip(OPT_HYPERS, (lr, beta1, beta2, 0.0))):
            t[f'optimizer/{h}' + VAR_SUFFIX] = np.array(val, np.float32)
    for n in NAMES:
        t[n + VAR_SUFFIX] = np.asarray(params[n], np.float32)
    if m is not None:
        for i, name in enumerate(METRICS):
            tot, cnt = (metrics or {}).get(name, (0.0, 0.0))
            t[f'keras_api/metrics/{i}/total' + VAR_SUFFIX] = np.array(tot, np.float32)
            t[f'keras_api/metrics/{i}/count' + VAR_SUFFIX] = np.array(cnt, np.float32)
        for s, src in (('m', m), ('v', v)):
            for n in NAMES:
                t[n + f'/.OPTIMIZER_SLOT/optimizer/{s}' + VAR_SUFFIX] = np.asarray(src[n], np.float32)
    t[OBJECT_GRAPH_KEY] = object_graph(t.keys())
    write_bundle(os.path.join(dest, 'variables', 'variables'), t,
                 shard_of=(lambda k: 0 if k == OBJECT_GRAPH_KEY else 1) if shards == 2 else None)
    from .savedmodel import saved_model_proto   # the SavedObjectGraph mirroring the object graph
    with open(os.path.join(dest, 'saved_model.pb'), 'wb') as fh:
        fh.write(saved_model_proto(t, V, d, reg=reg, lr=lr, beta1=beta1, beta2=beta2))
    json.dump({'num_cards': int(V), 'd': int(d), 'format': 'ccrec-mi355x/1'},
              open(os.path.join(dest, 'ccrec_config.json'), 'w'))


def load_variables(path):
    """Read ml_files/<name>/ -> (V, d, params dict, m dict|None, v dict|None, step)."""
    t = read_bundle(os.path.join(path, 'variables', 'variables'))
    if OBJECT_GRAPH_KEY in t:   # TF2 checkpoint: every variable the object graph names must be there
        for nd in parse_object_graph(t[OBJECT_GRAPH_KEY]):
            for _, _, key in nd['attrs']:
                if key not in t:
                    raise ValueError(f'{path}: object graph names {key!r}, absent from the bundle')
    params = {n: t[n + VAR_SUFFIX] for n in NAMES if n + VAR_SUFFIX in t}
    if 'encoder/encoded_1/kernel' not in params:
        raise ValueError(f'{path}: no encoder/encoded_1/kernel variable')
    V, d = params['encoder/encoded_1/kernel'].shape
    slot = lambda s: {n: t[n + f'/.OPTIMIZER_SLOT/optimizer/{s}' + VAR_SUFFIX] for n in NAMES
                      if n + f'/.OPTIMIZER_SLOT/optimizer/{s}' + VAR_SUFFIX in t}
    m, v = slot('m'), slot('v')
    step = int(t.get('optimizer/iter' + VAR_SUFFIX, np.array(0)))
    return int(V), int(d), params, (m or None), (v or None), step


def flat_params(path):
    V, d, params, m, v, step = load_variables(path)
    return V, d, Layout(V, d).pack(params)
