"""The oracle's hand-derived backward (oracle/model_ref.py) against torch-CPU autograd of the same
Keras forward and losses (float64): SURVEY §7.1's independent check of the gradients, the only one
available with TensorFlow absent.

Forward restated from the reference, not from the oracle: E = 4 ReLU Dense layers
(src/ml/model.py:27-42, the bottleneck included), D = 3 ReLU Dense + Dense(V) (:58-70), sigmoid for
D1 (:94) and softmax for D2 (:98) over E of one-hot reg rows (:117-125); loss = BCE + reg * KL
(src/ml/train.py:83-88) with TF 2.5's Keras semantics: BCE on a sigmoid output in logits form
(binary_crossentropy_with_logits, mean over V then B) and kullback_leibler_divergence with both
arguments clipped to [1e-7, 1] (clip's gradient passes inside the interval)."""
import numpy as np
import pytest
import torch

from oracle import model_ref


def _torch_loss(P, x_lists, y_lists, V, reg, reg_idx, y_reg):
    T = {k: torch.tensor(np.asarray(v, np.float64), requires_grad=True) for k, v in P.items()}
    B = len(x_lists)
    X = torch.zeros(B, V, dtype=torch.float64)
    Y = torch.zeros(B, V, dtype=torch.float64)
    for b in range(B):
        X[b, torch.as_tensor(np.asarray(x_lists[b], np.int64))] = 1
        Y[b, torch.as_tensor(np.asarray(y_lists[b], np.int64))] = 1

    def dense(h, name):
        return torch.relu(h @ T[name + '/kernel'] + T[name + '/bias'])

    def encoder(x):
        for n in ('encoded_1', 'encoded_2', 'encoded_3', 'bottleneck'):
            x = dense(x, 'encoder/' + n)
        return x

    def decoder(z, pre):
        for n in ('decoded_1', 'decoded_2', 'decoded_3'):
            z = dense(z, pre + '/' + n)
        return z @ T[pre + '/reconstruct/kernel'] + T[pre + '/reconstruct/bias']

    logits = decoder(encoder(X), 'decoder')
    bce = torch.nn.functional.binary_cross_entropy_with_logits(logits, Y, reduction='none').mean(1).mean()
    loss = bce
    kl = torch.zeros((), dtype=torch.float64)
    if reg > 0:
        I = torch.zeros(B, V, dtype=torch.float64)
        I[torch.arange(B), torch.as_tensor(np.asarray(reg_idx, np.int64))] = 1
        p = torch.softmax(decoder(encoder(I), 'decoder_for_reg'), dim=1)
        t = torch.clamp(torch.as_tensor(np.asarray(y_reg, np.float64)), 1e-7, 1.0)
        q = torch.clamp(p, 1e-7, 1.0)
        kl = (t * torch.log(t / q)).sum(1).mean()
        loss = bce + reg * kl
    loss.backward()
    G = {k: (v.grad.numpy() if v.grad is not None else np.zeros(tuple(v.shape))) for k, v in T.items()}
    return bce.item(), kl.item(), G


@pytest.mark.parametrize('reg', [0.0, 0.3])
@pytest.mark.parametrize('V,d,B', [(300, 64, 8), (517, 128, 5)])
def test_oracle_backward_equals_autograd(reg, V, d, B):
    rng = np.random.default_rng(V + B)
    P = model_ref.init_params(V, d, seed=V, bias_std=0.05)
    xs = [np.sort(rng.choice(V, int(rng.integers(3, 40)), replace=False)) for _ in range(B)]
    ys = [np.sort(rng.choice(x, max(1, len(x) - 2), replace=False)) for x in xs]
    reg_idx = rng.integers(0, V, B)
    y_reg = rng.dirichlet(np.ones(V) * 0.3, B)
    y_reg[y_reg < 1e-9] = 0.0            # zeros in the target rows (clip to 1e-7 applies)
    losses, G = model_ref.train_forward_backward(P, xs, ys, V, d, reg=reg, reg_idx=reg_idx,
                                                 y_reg=y_reg, mode='fp64')
    bce, kl, Gt = _torch_loss(P, xs, ys, V, reg, reg_idx, y_reg)
    assert abs(losses['bce'] - bce) <= 1e-12 * abs(bce)
    if reg > 0:
        assert abs(losses['kl'] - kl) <= 1e-12 * abs(kl)
    for k in P:
        if reg == 0 and k.startswith('decoder_for_reg'):
            continue
        a, b = np.asarray(G[k], np.float64), Gt[k]
        den = max(np.linalg.norm(b), 1e-300)
        assert np.linalg.norm(a - b) / den < 1e-10, k


def test_oracle_kl_clip_gradient_mask():
    """A regulariser row whose softmax has entries below 1e-7: the clipped entries pass no gradient
    through q (TF Maximum's mask), in the oracle and in autograd alike."""
    V, d, B = 200, 64, 3
    P = model_ref.init_params(V, d, seed=1, bias_std=0.0)
    P['decoder_for_reg/reconstruct/bias'] = np.linspace(-30, 8, V).astype(np.float32)  # tiny p's
    rng = np.random.default_rng(0)
    xs = [np.sort(rng.choice(V, 10, replace=False)) for _ in range(B)]
    reg_idx = np.array([0, 5, 199])
    y_reg = rng.dirichlet(np.ones(V), B)
    losses, G = model_ref.train_forward_backward(P, xs, xs, V, d, reg=1.0, reg_idx=reg_idx, y_reg=y_reg)
    _, _, Gt = _torch_loss(P, xs, xs, V, 1.0, reg_idx, y_reg)
    for k in ('decoder_for_reg/reconstruct/bias', 'decoder_for_reg/reconstruct/kernel',
              'encoder/encoded_1/kernel'):
        b = Gt[k]
        assert np.linalg.norm(G[k] - b) / np.linalg.norm(b) < 1e-10, k
