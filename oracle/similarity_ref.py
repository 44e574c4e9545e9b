"""Card similarity — ORACLE (test infrastructure only; never imported by the product path).

Reference: ``src/scripts/similarity.py:19-31``:
  embs  = model.encoder(identity [V, V])                 (encoder on every one-card row)
  dists = [CosineSimilarity()(embs[idx], x) for x in embs]
          Keras: -sum(l2_normalize(a) * l2_normalize(b)),  l2_normalize(x) = x * rsqrt(max(sum(x^2), 1e-12))
  ranked = dists.argsort();  prints ranked[:N] with their dists

Pinned arithmetic (identical on the GPU, ``cc_similar_cards``), float32, multiply and add separately
rounded, sums in index order: ss = sum_i e_i*e_i; inv = 1 / sqrt(max(ss, 1e-12)) (correctly rounded
sqrt and divide); dist = -(sum_i (q_i*inv_q) * (e_i*inv_e)).  Ranking: numpy
``argsort(dist, kind='stable')`` — ties (e.g. all-zero embeddings) by lower index first; the
reference's default argsort is unstable, so its tie order is implementation-defined.
TensorFlow's rsqrt is not restated bit-for-bit (TF is absent here): parity unpinned against TF.
"""
import numpy as np

from .infer_ref import DOT_CHUNK, TOWER

EPS = np.float32(1e-12)


def encode32_rows(P, rows):
    """infer_ref.encode32 for one-card rows, vectorised over the rows (same per-row arithmetic:
    a one-card E1 gather is 0 + W1[j], + 0, + b1; the Dense chunked sums as dense32)."""
    W1 = P['encoder/encoded_1/kernel']
    rows = np.asarray(rows, np.int64)
    zero = np.zeros((len(rows), W1.shape[1]), np.float32)
    part = (zero + W1[rows]).astype(np.float32)
    total = (zero + part).astype(np.float32)
    h = total + P['encoder/encoded_1/bias']
    h = np.where(h > 0, h, np.float32(0)).astype(np.float32)
    for nm in TOWER[:3]:
        Wk, b = P[nm + '/kernel'], P[nm + '/bias']
        K = Wk.shape[0]
        tot = np.zeros((len(rows), Wk.shape[1]), np.float32)
        for k0 in range(0, K, DOT_CHUNK):
            pt = np.zeros_like(tot)
            for k in range(k0, min(K, k0 + DOT_CHUNK)):
                pt = (pt + (h[:, k:k + 1] * Wk[k]).astype(np.float32)).astype(np.float32)
            tot = (tot + pt).astype(np.float32)
        h = (tot + b).astype(np.float32)
        h = np.where(h > 0, h, np.float32(0)).astype(np.float32)
    return h


def cosine_dists(emb, q):
    emb = np.asarray(emb, np.float32)
    K = emb.shape[1]
    qe = emb[q]
    ssq, sse = np.float32(0), np.zeros(len(emb), np.float32)
    for i in range(K):
        ssq = np.float32(ssq + np.float32(qe[i] * qe[i]))
        sse = (sse + (emb[:, i] * emb[:, i]).astype(np.float32)).astype(np.float32)
    invq = np.float32(np.float32(1) / np.sqrt(np.maximum(ssq, EPS)))
    inve = (np.float32(1) / np.sqrt(np.maximum(sse, EPS))).astype(np.float32)
    dot = np.zeros(len(emb), np.float32)
    for i in range(K):
        dot = (dot + (np.float32(qe[i] * invq) * (emb[:, i] * inve).astype(np.float32)).astype(np.float32)).astype(np.float32)
    return (-dot).astype(np.float32)


def most_similar(emb, q, N):
    d = cosine_dists(emb, q)
    order = np.argsort(d, kind='stable')[:N]
    return order, d[order], d
