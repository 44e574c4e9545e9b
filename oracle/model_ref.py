"""CC_Recommender forward/backward, Keras losses and TF Adam — ORACLE (test infra only).

Reference:
  * ``src/ml/model.py:20-48``  Encoder  E: Dense(d) -> Dense(256) -> Dense(128) -> Dense(64), all ReLU
    (the bottleneck has ReLU too, :33).  Reference width d = 512 (:27); build knob here.
  * ``src/ml/model.py:50-70``  Decoder  D: Dense(128) -> Dense(256) -> Dense(d) ReLU, then Dense(V)
    with sigmoid (D1, :94) or softmax (D2, :98).
  * ``src/ml/model.py:100-125`` call: (D1(E(x)), D2(E(identity rows))), one shared E.
  * ``src/ml/train.py:83-88`` compile(optimizer='adam', loss=[BCE, KL], loss_weights=[1, reg]).
TF 2.5.2 semantics restated (not vendored, not installed — "parity unpinned" vs TF itself):
  * BCE on a Sigmoid output = sigmoid_cross_entropy_with_logits: max(z,0) - z*y + log1p(exp(-|z|)),
    mean over V then over B; dL/dz = (sigmoid(z) - y) / (B*V).
  * KL: t = clip(y, 1e-7, 1), q = clip(p, 1e-7, 1), sum_j t log(t/q), mean over B; clip passes the
    gradient where p >= 1e-7 (Maximum/Minimum grads), softmax backward dz = p*(g - <p,g>).
  * ResourceApplyAdam: m += (g-m)(1-b1); v += (g^2-v)(1-b2);
    p -= lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps), lr=1e-3, b1=.9, b2=.999, eps=1e-7 (fp32).

``mode``: 'fp64' (exact reference), or 'bf16' which rounds exactly the operands the GPU's bf16
MFMA path rounds (weights' bf16 shadow, activations and dZ/dPre fed to GEMMs) while accumulating
in fp64 — the GPU's mixed-precision arithmetic up to summation order; 'mx8' is 'bf16' with the
decoder output-layer / regulariser products (model.py:64,94,98) on MX-FP8 operands exactly as
config 5 quantises them (oracle/mx8_ref.py: e4m3fn codes + one E8M0 scale per 32 K-elements, the
bf16 values quantised along each product's K axis), dequantised and accumulated in fp64.
"""
import numpy as np
import scipy.sparse as sp

TOWER_E = (256, 128, 64)
TOWER_D = (128, 256)


def layer_specs(V, d):
    """(name, fan_in, fan_out) in Keras creation order (model.py:27-33, 58-64, 92-98)."""
    enc = [('encoder/encoded_1', V, d), ('encoder/encoded_2', d, 256),
           ('encoder/encoded_3', 256, 128), ('encoder/bottleneck', 128, 64)]
    def dec(p):
        return [(p + '/decoded_1', 64, 128), (p + '/decoded_2', 128, 256),
                (p + '/decoded_3', 256, d), (p + '/reconstruct', d, V)]
    return enc + dec('decoder') + dec('decoder_for_reg')


def init_params(V, d, seed=0, bias_std=0.0):
    """Glorot-uniform kernels (Keras Dense default), zero (or N(0,bias_std)) biases, float32."""
    rng = np.random.default_rng(seed)
    P = {}
    for name, fi, fo in layer_specs(V, d):
        lim = np.sqrt(6.0 / (fi + fo))
        P[name + '/kernel'] = rng.uniform(-lim, lim, (fi, fo)).astype(np.float32)
        P[name + '/bias'] = (rng.normal(0, bias_std, fo) if bias_std else np.zeros(fo)).astype(np.float32)
    return P


def bf16_round(a):
    """Round-to-nearest-even to bfloat16, returned as float32 (no NaN handling needed)."""
    a = np.ascontiguousarray(a, np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    u = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) & np.uint64(0xFFFF0000)
    return u.astype(np.uint32).view(np.float32)


def _mx8_mm(A, B):
    """A [M, K] . B [N, K]^T on MX-FP8 operands quantised along K (config 5's block-scaled MFMA)."""
    from oracle import mx8_ref
    qa, sa = mx8_ref.quantize_rows(A)
    qb, sb = mx8_ref.quantize_rows(B)
    return mx8_ref.dequantize_rows(qa, sa) @ mx8_ref.dequantize_rows(qb, sb).T


def _rq(mode):
    if mode in ('bf16', 'mx8'):
        return lambda a: bf16_round(a).astype(np.float64)
    if mode == 'fp32':   # plain fp32 numpy (the CPU-baseline leg of bench.py)
        return lambda a: np.asarray(a, np.float32)
    return lambda a: np.asarray(a, np.float64)


def _csr(lists, V):
    indptr = np.zeros(len(lists) + 1, np.int64)
    indptr[1:] = np.cumsum([len(l) for l in lists])
    idx = np.concatenate([np.asarray(l, np.int64) for l in lists]) if len(lists) else np.zeros(0, np.int64)
    return sp.csr_matrix((np.ones(len(idx)), idx, indptr), shape=(len(lists), V))


def _relu(a):
    return np.where(a > 0, a, 0.0)


def train_forward_backward(P, x_lists, y_lists, V, d, reg=0.0, reg_idx=None, y_reg=None, mode='fp64'):
    """One Keras train_step's forward + backward (train.py:99-102 via model.py:117-125).

    x_lists / y_lists: per-cube sorted card lists of the noised input x and the target y.
    reg_idx [n] and y_reg [n, V] (rows of M~) are used when reg > 0: the regulariser rows, n = B
    sampled rows (generator.py:47-51) or all |V| identity rows (full mode, README.md:27); the KL
    is the mean over the n rows (Keras' batch mean), so its gradient carries reg / n.
    Returns (losses dict, grads dict keyed like P).
    """
    rq = _rq(mode)
    B = len(x_lists)
    bdt = np.float32 if mode == 'fp32' else np.float64
    W = {k: (rq(v) if k.endswith('/kernel') else np.asarray(v, bdt)) for k, v in P.items()}
    use_reg = reg > 0
    nreg = len(reg_idx) if use_reg else 0
    Xs = _csr(list(x_lists) + ([[int(i)] for i in reg_idx] if use_reg else []), V).astype(bdt)
    # E1: sparse gather-sum of the (bf16 shadow) rows + bias, ReLU
    pre1 = Xs @ W['encoder/encoded_1/kernel'] + W['encoder/encoded_1/bias']
    h1 = rq(_relu(pre1))
    acts = [h1]
    hs = h1
    for nm in ('encoder/encoded_2', 'encoder/encoded_3', 'encoder/bottleneck'):
        hs = rq(_relu(hs @ W[nm + '/kernel'] + W[nm + '/bias']))
        acts.append(hs)
    zlat = hs
    losses = {}
    grads = {k: np.zeros(v.shape, bdt) for k, v in P.items()}
    dzlat = np.zeros_like(zlat)

    def decoder_branch(prefix, rows, out_grad_fn):
        z_in = zlat[rows]
        hh = [z_in]
        h = z_in
        for nm in ('decoded_1', 'decoded_2', 'decoded_3'):
            h = rq(_relu(h @ W[prefix + '/' + nm + '/kernel'] + W[prefix + '/' + nm + '/bias']))
            hh.append(h)
        Wo = W[prefix + '/reconstruct/kernel']
        if mode == 'mx8':     # logits: D3 [rows][d] . Wo^T [V][d], both quantised along d
            z = _mx8_mm(h, Wo.T) + W[prefix + '/reconstruct/bias']
        else:
            z = h @ Wo + W[prefix + '/reconstruct/bias']
        loss, dz = out_grad_fn(z)
        dzq = rq(dz)
        if mode == 'mx8':     # dW: D3^T . dZ along the rows; dX: dZ . Wo^T along V
            grads[prefix + '/reconstruct/kernel'] += _mx8_mm(hh[3].T, dzq.T)
            dh = _mx8_mm(dzq, Wo)
        else:
            grads[prefix + '/reconstruct/kernel'] += hh[3].T @ dzq
            dh = dzq @ Wo.T
        grads[prefix + '/reconstruct/bias'] += dzq.sum(0)
        for li, nm in ((3, 'decoded_3'), (2, 'decoded_2'), (1, 'decoded_1')):
            dpre = rq(dh * (hh[li] > 0))
            grads[prefix + '/' + nm + '/kernel'] += hh[li - 1].T @ dpre
            grads[prefix + '/' + nm + '/bias'] += dpre.sum(0)
            dh = dpre @ W[prefix + '/' + nm + '/kernel'].T
        dzlat[rows] += dh
        return loss

    Y = _csr(y_lists, V).toarray().astype(bdt)

    def bce(z):
        l = np.maximum(z, 0) - z * Y + np.log1p(np.exp(-np.abs(z)))
        loss = l.mean(axis=1).mean()
        p = 1.0 / (1.0 + np.exp(-z))
        return loss, (p - Y) / (B * V)

    losses['bce'] = decoder_branch('decoder', np.arange(B), bce)
    if use_reg:
        T = np.clip(np.asarray(y_reg, np.float64), 1e-7, 1.0)

        def kl(z):
            zm = z - z.max(axis=1, keepdims=True)
            e = np.exp(zm)
            p = e / e.sum(axis=1, keepdims=True)
            q = np.clip(p, 1e-7, 1.0)
            loss = (T * np.log(T / q)).sum(axis=1).mean()
            g = np.where(p >= 1e-7, -T / q, 0.0)
            dz = p * (g - (p * g).sum(axis=1, keepdims=True))
            return loss, dz * (reg / nreg)

        losses['kl'] = decoder_branch('decoder_for_reg', np.arange(B, B + nreg), kl)
    else:
        losses['kl'] = 0.0
    losses['loss'] = losses['bce'] + reg * losses['kl']
    # encoder backward
    dh = dzlat
    names = ('encoder/encoded_1', 'encoder/encoded_2', 'encoder/encoded_3', 'encoder/bottleneck')
    for li in (3, 2, 1):
        dpre = rq(dh * (acts[li] > 0))
        grads[names[li] + '/kernel'] += acts[li - 1].T @ dpre
        grads[names[li] + '/bias'] += dpre.sum(0)
        dh = dpre @ W[names[li] + '/kernel'].T
    # fp32 on the GPU's fp32 path (exact row-scatter); the bf16 path's W1 gradient is a bf16
    # MFMA product (cc_embed_grad_mfma) whose B operand is dPre1 rounded to bf16, as for every
    # other Dense layer's dW
    dpre1 = rq(dh * (acts[0] > 0))
    grads['encoder/encoded_1/kernel'] += np.asarray(Xs.T @ dpre1)
    grads['encoder/encoded_1/bias'] += dpre1.sum(0)
    return losses, grads


def adam_tf(P, Mo, Vo, G, t, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7):
    """TF ResourceApplyAdam (training_ops ApplyAdam) in float32, local step t (1-based)."""
    f = np.float32
    b1p = np.power(f(beta1), f(t), dtype=np.float32)
    b2p = np.power(f(beta2), f(t), dtype=np.float32)
    alpha = f(lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p)
    for k in P:
        g = np.asarray(G[k], np.float32)
        m = Mo[k]
        v = Vo[k]
        m += (g - m) * (f(1) - f(beta1))
        v += (g * g - v) * (f(1) - f(beta2))
        P[k] -= (m * alpha) / (np.sqrt(v) + f(eps))
    return P, Mo, Vo


def forward_probs(P, cube_lists, V, d):
    """Plain fp64 D1(E(x)) for a batch of cubes (reference recommend math, any order)."""
    Xs = _csr(cube_lists, V)
    W = {k: np.asarray(v, np.float64) for k, v in P.items()}
    h = _relu(Xs @ W['encoder/encoded_1/kernel'] + W['encoder/encoded_1/bias'])
    for nm in ('encoder/encoded_2', 'encoder/encoded_3', 'encoder/bottleneck',
               'decoder/decoded_1', 'decoder/decoded_2', 'decoder/decoded_3'):
        h = _relu(h @ W[nm + '/kernel'] + W[nm + '/bias'])
    z = h @ W['decoder/reconstruct/kernel'] + W['decoder/reconstruct/bias']
    return 1.0 / (1.0 + np.exp(-z))
