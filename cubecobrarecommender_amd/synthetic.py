"""Synthetic cubes — there is no real data in this pipeline (data.zip is an LFS
pointer).  Popularity Zipf(s=1) over a random permutation of the cards; cube sizes
{180,360,450,540,720} with p={.05,.5,.15,.2,.1}; cards drawn without replacement ∝ popularity
(Gumbel top-k).  Generated on the GPU in chunks with a seeded torch generator (set-up plumbing,
not the timed hot path); returned as a CSR of sorted card ids.
"""
import numpy as np
import torch

SIZES = (180, 360, 450, 540, 720)
PROBS = (0.05, 0.5, 0.15, 0.2, 0.1)


def synthetic_cubes(C, V, seed=20250301, device='cuda', chunk=2048, sizes=SIZES, probs=PROBS):
    rng = np.random.default_rng(seed)
    pop = 1.0 / (1.0 + rng.permutation(V))
    n = rng.choice(np.asarray(sizes), size=C, p=np.asarray(probs)).astype(np.int64)
    logp = torch.from_numpy(np.log(pop).astype(np.float32)).to(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(int(seed))
    kmax = int(max(sizes))
    rows = []
    for c0 in range(0, C, chunk):
        c1 = min(C, c0 + chunk)
        u = torch.rand(c1 - c0, V, device=device, generator=gen).clamp_(1e-12, 1.0)
        g = logp[None, :] - torch.log(-torch.log(u))
        top = torch.topk(g, kmax, dim=1).indices          # descending perturbed log-popularity
        rows.append(top.to(torch.int32).cpu().numpy())
    top = np.concatenate(rows)
    indptr = np.zeros(C + 1, np.int64)
    indptr[1:] = np.cumsum(n)
    indices = np.empty(int(indptr[-1]), np.int32)
    for c in range(C):
        indices[indptr[c]:indptr[c + 1]] = np.sort(top[c, :n[c]])
    return indptr, indices


def neg_sampler_from_csr(indptr, indices, V):
    """generator.py:30 neg_sampler = colsum(M~)/sum(M~) for M~ from utils.py:75-91 + train.py:69-71,
    computed in O(nnz) without forming the V x V matrix:
        M~[i,j] = count[i,j] / S_i  with S_i = sum_{c ∋ i} |c|   (seen i),  e_i (never-seen i)
        colsum_j = sum_{c ∋ j} w_c + [j never seen],  w_c = sum_{i in c} 1 / S_i.
    Equal to the dense definition up to fp64 summation order (checked in tests/test_host.py)."""
    indptr = np.asarray(indptr, np.int64)
    indices = np.asarray(indices, np.int64)
    sizes = np.diff(indptr).astype(np.float64)
    cube_of = np.repeat(np.arange(len(sizes)), np.diff(indptr))
    S = np.bincount(indices, weights=sizes[cube_of], minlength=V)
    seen = S > 0
    inv = np.where(seen, 1.0 / np.where(seen, S, 1.0), 0.0)
    w = np.bincount(cube_of, weights=inv[indices], minlength=len(sizes))
    col = np.bincount(indices, weights=w[cube_of], minlength=V) + (~seen)
    return col / col.sum()
