"""Keras-shaped host mirror of ``src/ml/model.py`` / ``src/ml/train.py`` over the HIP hot path.

    model = CC_Recommender(num_cards)                                   # model.py:89-98
    model.compile(optimizer='adam', loss=['binary_crossentropy', 'kullback_leibler_divergence'],
                  loss_weights=[1.0, reg], metrics=['accuracy'])        # train.py:83-88
    model.fit(generator, epochs=epochs)                                # train.py:99-102
    model.save(dest, save_format='tf')                                  # train.py:112-115
    model = load_model(dest)                                            # ml_recommend.py:54
    model.decoder(model.encoder(x)).numpy()                             # ml_recommend.py:78-85

encoder/decoder run the fp32 pinned-order inference kernels (bit-exact vs oracle/infer_ref.py);
fit runs the device-resident training step (trainer.py) with TF Adam semantics.  There is no CPU
fallback: every compute call goes through libccrec_hip.so.
"""
import time

import numpy as np
import torch

from . import checkpoint
from .layout import Layout, glorot_flat
from .recommender import Recommender

_LOSSES = ('binary_crossentropy', 'kullback_leibler_divergence')
STATUS_EVERY = 16   # fit(): device status flags are read (one host sync) every this many steps


class Tensor:
    """What model.encoder(...) returns: supports .numpy() like a TF EagerTensor."""

    def __init__(self, t):
        self._t = t

    def numpy(self):
        return self._t.detach().cpu().numpy()

    def __array__(self, dtype=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def __getitem__(self, i):
        return Tensor(self._t[i])

    @property
    def shape(self):
        return tuple(self._t.shape)


def _rows_of(x):
    """Dense 0/1 input [R, V] (numpy/torch/Tensor) or a list of index lists -> list of index arrays."""
    if isinstance(x, Tensor):
        x = x.numpy()
    if isinstance(x, (list, tuple)) and (len(x) == 0 or not np.isscalar(x[0])):
        return [np.asarray(r, np.int64) for r in x]
    a = x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)
    if a.ndim == 1:
        a = a[None, :]
    return [np.nonzero(r == 1)[0] for r in a]


class _Encoder:
    def __init__(self, model):
        self.m = model

    def __call__(self, x, training=None):
        return Tensor(self.m._rec().encode_lists(_rows_of(x)))


class _Decoder:
    def __init__(self, model):
        self.m = model

    def __call__(self, z, training=None):
        zt = z._t if isinstance(z, Tensor) else torch.as_tensor(np.asarray(z, np.float32))
        return Tensor(self.m._rec().decode(zt))


class CC_Recommender:
    def __init__(self, num_cards, d=512, dtype='fp32', seed=0, params_flat=None):
        """dtype: GEMM operand precision of fit().  'fp32' (default) is the reference's precision
        (TF float32, model.py); 'bf16' (bf16 MFMA operands, fp32 master weights / Adam / losses) and
        'fp8' (+ MX-FP8 decoder output GEMMs) are opt-in."""
        self.N = int(num_cards)
        self.d = int(d)
        self.dtype = dtype
        self.seed = seed
        self.layout = Layout(self.N, self.d)
        self._flat = params_flat if params_flat is not None else glorot_flat(self.N, self.d, seed)
        self._m = self._v = None
        self._step = 0
        self._metrics = None
        self.metrics = []
        self.reg = 0.0
        self.lr = 1e-3
        self.trainer = None
        self._recommender = None
        self.encoder = _Encoder(self)
        self.decoder = _Decoder(self)
        self.history = []

    # --------------------------------------------------------------- Keras surface
    def compile(self, optimizer='adam', loss=_LOSSES, loss_weights=(1.0, 0.0), metrics=None,
                learning_rate=1e-3):
        if optimizer != 'adam':
            raise ValueError("only optimizer='adam' (train.py:84) is implemented")
        if tuple(loss) != _LOSSES:
            raise ValueError(f'loss must be {list(_LOSSES)} (train.py:85)')
        if float(loss_weights[0]) != 1.0:
            raise ValueError('loss_weights[0] must be 1.0 (train.py:86)')
        # metrics=['accuracy'] (train.py:87): TF 2.5 resolves it per output by shape
        # (compile_utils._get_metric_object: binary_accuracy only when y_pred's last dim is 1), so
        # both [B, |V|] outputs report categorical_accuracy, as epoch means over rows; fit() counts
        # both on the device (TrainConfig(metrics=True), metrics.hip).  They do not enter the loss,
        # the gradients or the update.
        self.metrics = []
        for mname in (metrics or ()):
            if mname not in ('accuracy', 'acc'):
                raise ValueError(f'metric {mname!r}: only the reference\'s metrics=[\'accuracy\'] is implemented')
            self.metrics = ['accuracy']
        self.reg = float(loss_weights[1])
        self.lr = float(learning_rate)

    def fit(self, generator, epochs=1, verbose=1, rank=0, world=1, graphs=True, log=print):
        """Keras ``fit(generator, epochs)`` (train.py:99-102).  The optimizer state persists across
        calls like Keras' (optimizer.iterations and the m/v slots): a second fit() resumes Adam's
        step count and moments, and the device step counter keeps the Philox noise draws fresh.
        The logged loss is the epoch mean over its batches, as Keras' progress bar reports it."""
        from .trainer import TrainConfig, Trainer
        cfg = TrainConfig(V=self.N, d=self.d, batch_size=generator.batch_size, reg=self.reg,
                          noise=generator.noise, noise_std=generator.noise_std, lr=self.lr,
                          dtype=self.dtype, seed=self.seed, rank=rank, world=world,
                          # one process: W1's Adam inside its gradient kernel and (BCE only) part of
                          # Wo's beside the tower backward chains, where the trainer's bf16 path
                          # supports it (bit-identical to the unfused step,
                          # tests/test_gpu_train.py::test_fused_w1_adam_matches_unfused) — the
                          # configuration bench.py measures
                          fuse_w1_adam=(world == 1), wo_adam_in_tower=(world == 1),
                          metrics=bool(self.metrics))
        tr = Trainer(cfg, generator.data, params_flat=self._current_flat())
        if self._m is not None:
            tr.load_standard(tr.m, self._m)
            tr.load_standard(tr.v, self._v)
            tr.state[0] = self._step
        tr.set_epoch_permutations(generator.epoch_permutations(epochs))
        steps = tr.batches_per_epoch
        loss_sum = torch.zeros(2, dtype=torch.float64, device=tr.loss_dev.device)
        if graphs:
            tr.capture(loss_acc=loss_sum)   # (one process: + the multi-step graph of step_many)
        for ep in range(epochs):
            t0 = time.perf_counter()
            loss_sum.zero_()
            i = 0
            while i < steps:
                # data-parallel: bucketed reduce-scatter + sharded Adam (zero.py) per step; one
                # process: multi-step graph replays; an x_cap / owner-capacity overflow stops the
                # run within STATUS_EVERY steps, not at epoch end
                n = min(STATUS_EVERY - i % STATUS_EVERY, steps - i)
                tr.step_many(n, loss_acc=loss_sum)
                i += n
                if i % STATUS_EVERY == 0:
                    tr.check_status()
            torch.cuda.synchronize()
            tr.check_status()
            l = tr.losses(loss_sum / steps)
            if world > 1:         # mean over ranks (each rank's loss is the mean over its cubes)
                t = torch.tensor([l['bce'], l['kl']], dtype=torch.float64, device=tr.loss_dev.device)
                torch.distributed.all_reduce(t)
                l = {'bce': float(t[0]) / world, 'kl': float(t[1]) / world}
                l['loss'] = l['bce'] + self.reg * l['kl']
            if tr.acc_counts is not None:   # Keras' history keys of the two outputs' accuracies
                l.update(tr.take_metrics(steps))
            self.history.append(l)
            # the compiled metrics' Mean accumulators as Keras leaves them after the epoch
            # (reset per epoch; update_state(value, sample_weight=batch)): 'loss' and the first
            # output's loss — written into the checkpoint with the optimizer state
            n = float(steps * cfg.batch_size * world)
            self._metrics = {'loss': (l['loss'] * n, n), 'output_1_loss': (l['bce'] * n, n)}
            if verbose and rank == 0:
                dt = time.perf_counter() - t0
                acc = ''.join(f' - {k}: {l[k]:.4f}' for k in ('output_1_accuracy', 'output_2_accuracy') if k in l)
                log(f'Epoch {ep + 1}/{epochs} - {steps} steps - {dt:.3f}s - loss: {l["loss"]:.6f} '
                    f'- bce: {l["bce"]:.6f} - kl: {l["kl"]:.6f}{acc} - {steps * cfg.batch_size * world / dt:.0f} cubes/s')

        tr.flush()
        if getattr(tr, 'sharded', None) is not None:   # data parallel: m, v are sharded — gather
            tr.sharded.gather_state()                   # them here, on every rank (collective)
        self._m = tr.standard(tr.m)
        self._v = tr.standard(tr.v)
        self.trainer = tr
        self._recommender = None
        self._step = int(tr.state[0].item())
        return self

    def save(self, dest, save_format='tf'):
        """model.save(dest, save_format='tf') (train.py:112-115).  No collectives: fit() already
        gathered the optimizer state, so a data-parallel run may save from rank 0 alone."""
        lay = self.layout
        P = lay.unpack(self._current_flat())
        if self._m is not None:
            m, v = lay.unpack(self._m), lay.unpack(self._v)
        else:
            m = v = None
        checkpoint.save_model(dest, self.N, self.d, P, m, v, step=self._step, lr=self.lr, metrics=self._metrics,
                              reg=self.reg)

    # --------------------------------------------------------------- internals
    def _current_flat(self):
        if self.trainer is not None:
            return self.trainer.standard(self.trainer.params)
        return np.asarray(self._flat, np.float32)

    def _rec(self):
        if self._recommender is None:
            self._recommender = Recommender(self._current_flat(), self.N, self.d)
        return self._recommender

    def recommender(self):
        """The resident single-cube recommend engine (fp32 forward + GPU top-N)."""
        return self._rec()


def load_model(path, dtype='fp32'):
    """keras.models.load_model('ml_files/<name>') (ml_recommend.py:54, ml_recommend_web.py:37)."""
    V, d, params, m, v, step = checkpoint.load_variables(path)
    lay = Layout(V, d)
    model = CC_Recommender(V, d=d, dtype=dtype, params_flat=lay.pack(params))
    if m is not None and v is not None:
        model._m, model._v = lay.pack(m), lay.pack(v)
    model._step = step
    return model
