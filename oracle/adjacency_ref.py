"""Conditional-probability graph M and its row-normalised form M~ — ORACLE (test infra only).

``adjacency`` restates ``src/non_ml/utils.py:75-91`` (create_adjacency_matrix):
    M[i, j] = |{cubes containing i and j}| / |{cubes containing i}|, rows of never-seen
    cards stay all-zero (:85-88); optional ``force_diag`` (:90-91).
``normalise`` restates ``src/ml/train.py:69-71``:
    M~ = (M with diag := 1) / rowsum  (a never-seen row becomes e_i).
Both are pinned against the reference's own ``create_adjacency_matrix`` output in
``tests/golden/adjacency_*.npz``.
"""
import numpy as np


def adjacency(cubes_dense, force_diag=None):
    """M from a dense 0/1 cube matrix [C, V] (float64), via co-occurrence counts.

    counts = X^T X (exact integers in float64), M[i] = counts[i] / counts[i, i] when
    counts[i, i] != 0, else counts[i] (all zeros) — utils.py:82-89.
    """
    X = np.asarray(cubes_dense, np.float64)
    counts = X.T @ X
    diag = np.diag(counts).copy()
    out = np.where(diag[:, None] != 0, counts / np.where(diag == 0, 1.0, diag)[:, None], counts)
    if force_diag is not None:
        np.fill_diagonal(out, force_diag)
    return out


def adjacency_from_lists(cube_lists, num_cards):
    X = np.zeros((len(cube_lists), num_cards))
    for c, lst in enumerate(cube_lists):
        X[c, np.asarray(lst, np.int64)] = 1
    return adjacency(X)


def normalise(adj_mtx):
    """train.py:69-71."""
    y = np.array(adj_mtx, dtype=np.float64, copy=True)
    np.fill_diagonal(y, 1)
    return y / y.sum(1)[:, None]
