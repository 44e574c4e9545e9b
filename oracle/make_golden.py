"""Generate golden vectors by running the REFERENCE's own numpy code (this container only).

ORACLE tooling — test infrastructure only.  Imports, read-only, from /root/reference:
  * ``src/non_ml/utils.py``    (create_adjacency_matrix, utils.py:75-91) — imports numpy/json/os only;
  * ``src/ml/generator.py``    (DataGenerator, generator.py:4-103) — it only *subclasses*
    ``tensorflow.keras.utils.Sequence`` (generator.py:1,4); TensorFlow is not installed, so an
    empty base class is registered under that module name for the import.
Nothing from the reference is copied: the outputs (inputs + expected outputs) are written as
small ``.npz`` fixtures under ``tests/golden/``; the reference never travels to the GPU box.

Run:  python -m oracle.make_golden [case ...]   (from the repo root; no case: all of them)
"""
import os
import sys
import types

import numpy as np

REF = '/root/reference'
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')


def _import_reference():
    sys.dont_write_bytecode = True
    tf = types.ModuleType('tensorflow')
    keras = types.ModuleType('tensorflow.keras')
    kutils = types.ModuleType('tensorflow.keras.utils')

    class Sequence:  # generator.py only subclasses it
        pass

    kutils.Sequence = Sequence
    tf.keras = keras
    keras.utils = kutils
    sys.modules.setdefault('tensorflow', tf)
    sys.modules.setdefault('tensorflow.keras', keras)
    sys.modules.setdefault('tensorflow.keras.utils', kutils)
    sys.path.insert(0, os.path.join(REF, 'src', 'non_ml'))
    sys.path.insert(0, os.path.join(REF, 'src', 'ml'))
    import utils as ref_utils  # noqa: E402
    import generator as ref_generator  # noqa: E402
    return ref_utils, ref_generator


def synthetic_dense_cubes(rng, C, V, sizes, never_seen=2):
    """Zipf-popular cubes (SURVEY §8(d) recipe at small scale); the last ``never_seen`` cards never
    appear, exercising the all-zero rows of utils.py:85-88 / e_i rows of train.py:69-71."""
    live = V - never_seen
    pop = 1.0 / (1.0 + rng.permutation(live))
    X = np.zeros((C, V))
    for c in range(C):
        n = int(rng.choice(sizes))
        g = np.log(pop) + rng.gumbel(size=live)
        X[c, np.argsort(-g)[:n]] = 1
    return X


def normalise(adj):
    # train.py:69-71 (train.py executes at import time, so the three lines are applied here)
    y = adj.copy()
    np.fill_diagonal(y, 1)
    return y / y.sum(1)[:, None]


def main():
    ref_utils, ref_gen = _import_reference()
    os.makedirs(OUT, exist_ok=True)
    cases = [
        # name, seed, C, V, sizes, B, batches
        ('small', 20250301, 48, 120, (6, 12, 20, 30), 8, 3),
        ('medium', 7, 160, 900, (40, 90, 140, 200), 32, 2),
        # the bench's kernel class (bf16, d = 256, B = 128: the fused output-layer kernels) on the
        # reference generator's own batches; M is not stored (50 MB), its oracle is pinned above
        ('bench', 11, 512, 2500, (20, 40, 80), 128, 2),
    ]
    only = sys.argv[1:]
    for name, seed, C, V, sizes, B, nb in cases:
        if only and name not in only:
            continue
        rng = np.random.default_rng(seed)
        X = synthetic_dense_cubes(rng, C, V, sizes)
        M = ref_utils.create_adjacency_matrix(X, verbose=False)
        Mt = normalise(M)
        # generator: global legacy MT19937 seeded exactly as train.py:20-25 would
        np.random.seed(seed % (2 ** 32))
        gen = ref_gen.DataGenerator(Mt, X, batch_size=B, noise=0.2, noise_std=0.1)
        perm0 = gen.indices.copy()
        xs, ys, regs, perms = [], [], [], []
        for bi in range(nb):
            (xc, xr), (yc, yr) = gen[bi]
            assert np.array_equal(yr, Mt[np.argmax(xr, axis=1)])
            xs.append(xc.astype(np.int8))
            ys.append(yc.astype(np.int8))
            regs.append(np.argmax(xr, axis=1))
        gen.on_epoch_end()
        perm1 = gen.indices.copy()
        (xc, xr), (yc, yr) = gen[0]
        xs.append(xc.astype(np.int8))
        ys.append(yc.astype(np.int8))
        regs.append(np.argmax(xr, axis=1))
        np.savez_compressed(
            os.path.join(OUT, f'generator_{name}.npz'),
            seed=np.int64(seed % (2 ** 32)), cubes=X.astype(np.int8), B=np.int64(B),
            neg_sampler=gen.neg_sampler, perm0=perm0, perm1=perm1,
            x=np.stack(xs), y=np.stack(ys), reg=np.stack(regs))
        if name != 'bench':
            np.savez_compressed(os.path.join(OUT, f'adjacency_{name}.npz'),
                                cubes=X.astype(np.int8), M=M, Mt=Mt)
        print(name, 'C', C, 'V', V, 'batches', len(xs), 'M nnz', int((M > 0).sum()))


if __name__ == '__main__':
    main()
