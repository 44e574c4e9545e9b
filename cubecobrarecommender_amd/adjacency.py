"""Conditional-probability graph M (src/non_ml/utils.py:75-91) and M~ (src/ml/train.py:69-71).

Set-up path (not the timed hot path): counts = X^T X for the 0/1 cube matrix X, computed on the
GPU in fp32 (exact: counts < 2^24) in row chunks of cubes; M[i] = counts[i] / counts[i,i] (rows of
never-seen cards stay 0), then M~ = (M with diag := 1) / rowsum.  A hand-written binary-GEMM
kernel for this is SURVEY §8(f) row N1 ("next").
"""
import numpy as np
import torch


def cooccurrence_gpu(indptr, indices, V, device='cuda', chunk=8192):
    indptr = np.asarray(indptr, np.int64)
    C = len(indptr) - 1
    counts = torch.zeros(V, V, device=device, dtype=torch.float32)
    for c0 in range(0, C, chunk):
        c1 = min(C, c0 + chunk)
        X = torch.zeros(c1 - c0, V, device=device, dtype=torch.float32)
        rows = np.repeat(np.arange(c1 - c0), np.diff(indptr[c0:c1 + 1]))
        cols = indices[indptr[c0]:indptr[c1]]
        X[torch.from_numpy(rows).to(device), torch.from_numpy(np.asarray(cols, np.int64)).to(device)] = 1.0
        counts.addmm_(X.t(), X)
    return counts


def adjacency_normalised_gpu(indptr, indices, V, device='cuda'):
    counts = cooccurrence_gpu(indptr, indices, V, device)
    diag = torch.diagonal(counts).clone()
    M = torch.where(diag[:, None] != 0, counts / torch.where(diag == 0, 1.0, diag)[:, None], counts)
    del counts
    M.fill_diagonal_(1.0)
    M /= M.sum(1, keepdim=True)
    return M
