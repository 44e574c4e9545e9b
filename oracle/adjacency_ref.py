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


def normalised_rows_from_lists(cube_lists, num_cards, rows):
    """Rows ``rows`` of M~ (utils.py:75-91 then train.py:69-71) without forming the V x V matrix:
    for each requested card i, counts[i, :] over the cubes containing i, M[i] = counts[i] / d_i
    (all-zero when d_i = 0), diagonal := 1, divided by the row sum — the same float64 operations
    as ``normalise(adjacency_from_lists(...))`` restricted to those rows."""
    V = int(num_cards)
    rows = np.asarray(rows, np.int64)
    holders = {}
    for c, lst in enumerate(cube_lists):
        for j in np.unique(np.asarray(lst, np.int64)):
            holders.setdefault(int(j), []).append(c)
    out = np.zeros((len(rows), V))
    cache = {}
    for r, i in enumerate(rows):
        i = int(i)
        if i not in cache:
            counts = np.zeros(V)
            for c in holders.get(i, ()):
                counts[np.unique(np.asarray(cube_lists[c], np.int64))] += 1.0
            d = counts[i]
            m = counts / d if d != 0 else counts
            m[i] = 1.0
            cache[i] = m / m.sum()
        out[r] = cache[i]
    return out
