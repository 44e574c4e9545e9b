"""Recommend forward pass + top-N with a pinned fp32 order — ORACLE (test infrastructure only).

Reference: ``src/scripts/ml_recommend.py:78-108`` and ``web/ml_recommend_web.py:39-64``:
  results = decoder(encoder(cube[1,V]))[0]   (fp32 Keras inference)
  ranked  = results.argsort()[::-1]
  additions = first ``amount`` of ranked not in the cube (the loop adds before testing
              ``recommended >= amount``, so amount <= 0 still yields one addition, :94-104)
  cuts      = {card: results[idx] for idx in cube_indices}  (:106-108)

Pinned arithmetic (identical on the GPU, ``cc_infer_fwd_fp32``), all fp32, multiply and add
separately rounded (no FMA):
  * E1 gather: the cube's sorted unique indices in chunks of GATHER_CHUNK consecutive entries;
    each chunk summed sequentially from 0; chunk sums added sequentially from 0; then + bias.
  * every Dense dot product: K split into chunks of DOT_CHUNK; each chunk acc = acc + h[k]*W[k,c]
    from 0; chunk partials added sequentially from 0; then + bias; ReLU as (x > 0 ? x : 0).
  * sigmoid: float32(1 / (1 + exp(-z))) in float64 with the deterministic exp (detmath.py).
  * ranking: numpy ``argsort(kind='stable')[::-1]`` — descending value, ties by higher index first
    (the reference's default argsort is unstable, so its tie order is implementation-defined).
"""
import numpy as np

from .detmath import det_sigmoid32

GATHER_CHUNK = 32
DOT_CHUNK = 64

TOWER = ('encoder/encoded_2', 'encoder/encoded_3', 'encoder/bottleneck',
         'decoder/decoded_1', 'decoder/decoded_2', 'decoder/decoded_3')


def _relu32(a):
    return np.where(a > 0, a, np.float32(0)).astype(np.float32)


def gather_e1(W1, b1, idx):
    idx = np.unique(np.asarray(idx, np.int64))
    d = W1.shape[1]
    total = np.zeros(d, np.float32)
    for c0 in range(0, len(idx), GATHER_CHUNK):
        part = np.zeros(d, np.float32)
        for j in idx[c0:c0 + GATHER_CHUNK]:
            part = (part + W1[j]).astype(np.float32)
        total = (total + part).astype(np.float32)
    return _relu32(total + b1)


def dense32(h, Wk, b, relu=True):
    h = np.asarray(h, np.float32)
    Wk = np.asarray(Wk, np.float32)
    K = Wk.shape[0]
    total = np.zeros(Wk.shape[1], np.float32)
    for k0 in range(0, K, DOT_CHUNK):
        part = np.zeros(Wk.shape[1], np.float32)
        for k in range(k0, min(K, k0 + DOT_CHUNK)):
            part = (part + (h[k] * Wk[k]).astype(np.float32)).astype(np.float32)
        total = (total + part).astype(np.float32)
    out = (total + np.asarray(b, np.float32)).astype(np.float32)
    return _relu32(out) if relu else out


def encode32(P, idx):
    h = gather_e1(P['encoder/encoded_1/kernel'], P['encoder/encoded_1/bias'], idx)
    for nm in TOWER[:3]:
        h = dense32(h, P[nm + '/kernel'], P[nm + '/bias'])
    return h


def decode32(P, zlat):
    h = zlat
    for nm in TOWER[3:]:
        h = dense32(h, P[nm + '/kernel'], P[nm + '/bias'])
    z = dense32(h, P['decoder/reconstruct/kernel'], P['decoder/reconstruct/bias'], relu=False)
    return det_sigmoid32(z)


def recommend_probs(P, idx):
    return decode32(P, encode32(P, idx))


def rank(results):
    return np.argsort(np.asarray(results, np.float32), kind='stable')[::-1]


def top_n(results, cube_indices, amount):
    """ml_recommend.py:94-108 with the pinned tie rule; returns (additions idx array, cut idx list)."""
    in_cube = np.zeros(len(results), bool)
    in_cube[np.asarray(cube_indices, np.int64)] = True
    order = rank(results)
    cand = order[~in_cube[order]]
    n_add = max(int(amount), 1)
    return cand[:n_add], list(cube_indices)
