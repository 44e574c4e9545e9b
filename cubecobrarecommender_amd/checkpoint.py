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

The writer produces a bundle any tensor-bundle reader (tf.train.load_checkpoint) can parse; the
reader parses such files (multi-block, prefix-compressed, multi-shard).  ``saved_model.pb`` (the
TF graph, which TF is needed to produce) is written as an empty SavedModel message, and
``ccrec_config.json`` records (V, d).  No real checkpoint exists in this pipeline (all ml_files
are Git-LFS pointers), so compatibility with files written by TF itself is unpinned.
"""
import json
import os
import struct

import numpy as np

from . import _lib as L
from .layout import NAMES, Layout

MAGIC = 0xdb4775248b80fb57
DT_FLOAT, DT_INT64 = 1, 9
_NP = {DT_FLOAT: np.float32, DT_INT64: np.int64}
VAR_SUFFIX = '/.ATTRIBUTES/VARIABLE_VALUE'


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
def _block(entries):
    """LevelDB block, restart at every entry (no prefix sharing): valid for any reader."""
    out = bytearray()
    restarts = []
    for k, v in entries:
        restarts.append(len(out))
        out += _varint(0) + _varint(len(k)) + _varint(len(v)) + k + v
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack('<I', r)
    out += struct.pack('<I', len(restarts))
    return bytes(out)


def _write_table(path, entries):
    entries = sorted(entries, key=lambda kv: kv[0])
    f = bytearray()

    def put_block(data):
        off = len(f)
        f.extend(data)
        f.append(0)                                   # no compression
        f.extend(struct.pack('<I', _mask(crc32c(data + b'\x00'))))
        return off, len(data)

    d_off, d_len = put_block(_block(entries))
    m_off, m_len = put_block(_block([]))
    last = entries[-1][0] if entries else b''
    i_off, i_len = put_block(_block([(last, _varint(d_off) + _varint(d_len))]))
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
def write_bundle(prefix, tensors):
    """tensors: dict key -> numpy array (float32 / int64).  Writes <prefix>.index + .data-00000-of-00001."""
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    entries = [(b'', _header_proto(1))]
    off = 0
    with open(prefix + '.data-00000-of-00001', 'wb') as fh:
        for key in sorted(tensors):
            a = np.array(tensors[key], order="C", copy=True)   # keeps 0-d scalars 0-d
            dt = DT_FLOAT if a.dtype == np.float32 else DT_INT64
            a = a.astype(_NP[dt], copy=False)
            raw = a.tobytes()
            fh.write(raw)
            entries.append((key.encode(), _entry_proto(dt, a.shape, 0, off, len(raw), _mask(crc32c(raw)))))
            off += len(raw)
    _write_table(prefix + '.index', entries)


def read_bundle(prefix, verify=True):
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
        if dt not in _NP:
            continue
        shape = [(_parse(dim).get(1, [0])[0]) for dim in _parse(e[2][0]).get(2, [])] if 2 in e else []
        shard, off, size = e.get(3, [0])[0], e.get(4, [0])[0], e.get(5, [0])[0]
        raw = np.asarray(shards[shard][off:off + size])
        if verify and 6 in e and _unmask(e[6][0]) != crc32c(raw):
            raise ValueError(f'crc mismatch for {k!r}')
        out[k.decode()] = raw.view(_NP[dt]).reshape(shape).copy()
    return out


# ---------------------------------------------------------------------------- model files
def save_model(dest, V, d, params, m=None, v=None, step=0, lr=1e-3, beta1=0.9, beta2=0.999):
    """ml_files/<name>/ as train.py:112-115 lays it out.  params/m/v: dict name -> array."""
    os.makedirs(os.path.join(dest, 'variables'), exist_ok=True)
    t = {}
    for n in NAMES:
        t[n + VAR_SUFFIX] = np.asarray(params[n], np.float32)
        if m is not None:
            t[n + '/.OPTIMIZER_SLOT/optimizer/m' + VAR_SUFFIX] = np.asarray(m[n], np.float32)
            t[n + '/.OPTIMIZER_SLOT/optimizer/v' + VAR_SUFFIX] = np.asarray(v[n], np.float32)
    if m is not None:
        t['optimizer/iter' + VAR_SUFFIX] = np.array(step, np.int64)
        t['optimizer/learning_rate' + VAR_SUFFIX] = np.array(lr, np.float32)
        t['optimizer/beta_1' + VAR_SUFFIX] = np.array(beta1, np.float32)
        t['optimizer/beta_2' + VAR_SUFFIX] = np.array(beta2, np.float32)
        t['optimizer/decay' + VAR_SUFFIX] = np.array(0.0, np.float32)
    write_bundle(os.path.join(dest, 'variables', 'variables'), t)
    open(os.path.join(dest, 'saved_model.pb'), 'wb').close()          # empty SavedModel message
    json.dump({'num_cards': int(V), 'd': int(d), 'format': 'ccrec-mi355x/1'},
              open(os.path.join(dest, 'ccrec_config.json'), 'w'))


def load_variables(path):
    """Read ml_files/<name>/ -> (V, d, params dict, m dict|None, v dict|None, step)."""
    t = read_bundle(os.path.join(path, 'variables', 'variables'))
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
