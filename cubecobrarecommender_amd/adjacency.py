"""Card co-occurrence graph on the GPU — SURVEY §8(f) row N1.

Replaces ``create_adjacency_matrix`` (src/non_ml/utils.py:75-91, run by
src/non_ml/create_mtx.py:19) and the M~ normalisation of src/ml/train.py:69-71 with one C-ABI
call, ``cc_adjacency`` (csrc/cooccur.hip): an FP4 (MX-scaled) MFMA GEMM of the transposed 0/1 cube matrix
with itself (exact counts, upper-triangle tiles only) whose epilogue writes

    counts  int32  |{cubes containing i and j}|
    M       f64    counts[i, j] / counts[i, i]; rows of unseen cards 0; diag := force_diag
                   (bit-exact with the reference's f64 M — the output/full_adj_mtx.npy format)
    M~      f32    (M with diag := 1) / rowsum; an unseen card's row is e_i

Cubes are CSR lists (``indptr``, ``indices``) instead of the reference's dense [C, V] f64
matrix; ``dense_to_csr`` converts one.  There is no CPU fallback: the HIP library must load.
"""
import numpy as np
import torch

from . import _lib


def dense_to_csr(cubes):
    """Dense 0/1 cube matrix [C, V] (the reference's utils.build_cubes output) -> CSR lists."""
    cubes = np.asarray(cubes)
    rows, cols = np.nonzero(cubes)
    indptr = np.zeros(cubes.shape[0] + 1, np.int64)
    np.add.at(indptr, rows + 1, 1)
    return np.cumsum(indptr), cols.astype(np.int32)


def _device_lists(indptr, indices, V, device):
    indptr = np.asarray(indptr, np.int64)
    indices = np.asarray(indices, np.int64)
    if indptr.ndim != 1 or len(indptr) < 1 or indptr[0] != 0 or np.any(np.diff(indptr) < 0):
        raise ValueError('indptr must start at 0 and be non-decreasing')
    if indptr[-1] != len(indices):
        raise ValueError('indptr[-1] must equal len(indices)')
    if len(indices) >= 2 ** 31:
        raise ValueError('too many (cube, card) entries for int32 offsets')
    if len(indices) and (indices.min() < 0 or indices.max() >= V):
        raise IndexError(f'card id out of range [0, {V})')   # the reference's IndexError
    rp = torch.from_numpy(indptr.astype(np.int32)).to(device)
    ix = torch.from_numpy(indices.astype(np.int32)).to(device) if len(indices) else \
        torch.zeros(1, dtype=torch.int32, device=device)
    return rp, ix, len(indptr) - 1


def upload_lists(indptr, indices, V, device='cuda'):
    """Validate CSR cube lists on the host and copy them to the device (int32)."""
    return _device_lists(indptr, indices, int(V), device)


def adjacency_device(rp, ix, C, V, outputs=('M',), force_diag=None, chunk_cubes=0, stream=None):
    """cc_adjacency on already-uploaded lists (see upload_lists); returns device tensors."""
    outputs = set(outputs)
    if not outputs or not outputs <= {'counts', 'M', 'Mt'}:
        raise ValueError("outputs must be a non-empty subset of {'counts', 'M', 'Mt'}")
    V = int(V)
    if V <= 0:
        raise ValueError('V must be positive')
    device = rp.device
    L = _lib.lib()
    with_counts = 'counts' in outputs
    ws_bytes = L.cc_adjacency_ws_size(V, C, int(chunk_cubes), int(with_counts))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
    out = {}
    if with_counts:
        out['counts'] = torch.empty(V, V, dtype=torch.int32, device=device)
    if 'M' in outputs:
        out['M'] = torch.empty(V, V, dtype=torch.float64, device=device)
    if 'Mt' in outputs:
        out['Mt'] = torch.empty(V, V, dtype=torch.float32, device=device)
    fd = _lib.C.byref(_lib.C.c_double(float(force_diag))) if force_diag is not None else None
    _lib.check(L.cc_adjacency(_lib.ptr(rp), _lib.ptr(ix), C, V, int(chunk_cubes), fd,
                              _lib.ptr(ws), _lib.ptr(out.get('counts')), _lib.ptr(out.get('M')),
                              _lib.ptr(out.get('Mt')), _lib.stream_ptr(stream)), 'cc_adjacency')
    del ws   # stream-ordered reuse by the caching allocator is safe
    return out


def adjacency_gpu(indptr, indices, V, outputs=('M',), force_diag=None, chunk_cubes=0,
                  device='cuda', stream=None):
    """Returns a dict with the requested outputs among 'counts', 'M', 'Mt' (device tensors)."""
    if int(V) <= 0:
        raise ValueError('V must be positive')
    rp, ix, C = upload_lists(indptr, indices, V, device)
    return adjacency_device(rp, ix, C, V, outputs, force_diag, chunk_cubes, stream)


def create_adjacency_matrix(cubes, verbose=False, force_diag=None, device='cuda'):
    """Drop-in for utils.create_adjacency_matrix(cubes, verbose, force_diag) (utils.py:75):
    dense [C, V] 0/1 cubes in, f64 numpy M out (computed on the GPU)."""
    indptr, indices = dense_to_csr(cubes)
    M = adjacency_gpu(indptr, indices, np.asarray(cubes).shape[1], ('M',), force_diag,
                      device=device)['M']
    return M.cpu().numpy()


def adjacency_normalised_gpu(indptr, indices, V, device='cuda', chunk_cubes=0):
    """M~ (fp32, [V, V], on the device) — the D2 regularisation target (train.py:69-71)."""
    return adjacency_gpu(indptr, indices, V, ('Mt',), chunk_cubes=chunk_cubes, device=device)['Mt']
