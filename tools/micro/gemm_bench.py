"""Time the decoder GEMM shapes through cc_gemm (dev tool).  Run under rocprofv3 --stats for
per-kernel durations; prints torch-event averages per variant."""
import ctypes as C
import sys

import torch

sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402

B, V, d, SPL = 512, 22000, 256, 16
dev = 'cuda'
bf = dict(device=dev, dtype=torch.bfloat16)
D3 = torch.randn(B, d, **bf)
D3t = D3.t().contiguous()
WoT = (torch.randn(V, d, **bf) * 0.05)
Wo = WoT.t().contiguous()
dZ = torch.randn(B, V, **bf) * 1e-4
dZt = dZ.t().contiguous()
bias = torch.zeros(V, device=dev)
ybits = torch.randint(0, 2**31 - 1, (B, (V + 31) // 32), device=dev, dtype=torch.int32)
part = torch.zeros(4096, device=dev, dtype=torch.float64)
Cb = torch.empty(B, V, **bf)
Ct = torch.empty(V, B, **bf)
gW = torch.empty(d, V, device=dev)
gb = torch.empty(V, device=dev)
split = torch.empty(64 * B * d, device=dev)


def gemm(M, N, K, A, lda, Bp, ldb, epi, **kw):
    g = L.GemmArgs()
    g.dtype, g.ta, g.tb, g.epilogue = L.CC_BF16, 0, 1, epi
    g.M, g.N, g.K, g.lda, g.ldb, g.ldc, g.splits, g.relu = M, N, K, lda, ldb, kw.get('ldc', N), kw.get('splits', 1), 0
    g.A, g.B = A.data_ptr(), Bp.data_ptr()
    for k in ('bias', 'C', 'Cf', 'y_bits', 'loss_partials', 'colsum', 'Ct'):
        v = kw.get(k)
        setattr(g, k, v.data_ptr() if v is not None else None)
    g.scale = 1.0 / (B * V)
    g.ldct = kw.get('ldct', 0)
    L.call('cc_gemm', C.byref(g), L.stream_ptr())


def main(only=None):
    variants = {
        'bce+C+Ct': lambda: gemm(B, V, d, D3, d, WoT, d, L.CC_EPI_BCE, bias=bias, C=Cb, y_bits=ybits,
                                 loss_partials=part, Ct=Ct, ldct=B),
        'bce+C': lambda: gemm(B, V, d, D3, d, WoT, d, L.CC_EPI_BCE, bias=bias, C=Cb, y_bits=ybits,
                              loss_partials=part),
        'store_bf16': lambda: gemm(B, V, d, D3, d, WoT, d, L.CC_EPI_STORE, C=Cb),
        'compute_only': lambda: gemm(B, V, d, D3, d, WoT, d, L.CC_EPI_STORE),
        'dW+colsum': lambda: gemm(d, V, B, D3t, B, dZt, B, L.CC_EPI_STORE, Cf=gW, colsum=gb),
        'dX_splitk': lambda: gemm(B, d, V, dZ, V, Wo, V, L.CC_EPI_SPLITK, Cf=split, splits=SPL),
        'dX_splitk8': lambda: gemm(B, d, V, dZ, V, Wo, V, L.CC_EPI_SPLITK, Cf=split, splits=8),
        'dX_splitk32': lambda: gemm(B, d, V, dZ, V, Wo, V, L.CC_EPI_SPLITK, Cf=split, splits=32),
        'dX_splitk64': lambda: gemm(B, d, V, dZ, V, Wo, V, L.CC_EPI_SPLITK, Cf=split, splits=64),
        'reduce16': lambda: L.call('cc_splitk_reduce', L.CC_BF16, L.ptr(split), 16, B, d, None, L.ptr(Cb), None, None, None, L.stream_ptr()),
        'reduce32': lambda: L.call('cc_splitk_reduce', L.CC_BF16, L.ptr(split), 32, B, d, None, L.ptr(Cb), None, None, None, L.stream_ptr()),
        'reduce64': lambda: L.call('cc_splitk_reduce', L.CC_BF16, L.ptr(split), 64, B, d, None, L.ptr(Cb), None, None, None, L.stream_ptr()),
    }
    for name, fn in variants.items():
        if only and name != only:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f'{name:14s} {e0.elapsed_time(e1) / 50 * 1000:8.1f} us', flush=True)

    if only:
        return
    # steady-state reference shapes (compute only)
    for (M, N, K) in ((512, 22016, 2048), (4096, 4096, 4096), (512, 22016, 256)):
        A = torch.randn(M, K, **bf)
        Bt = torch.randn(N, K, **bf)
        fn = lambda: gemm(M, N, K, A, K, Bt, K, L.CC_EPI_STORE)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1000
        print(f'{M}x{N}x{K} compute-only {us:8.1f} us  {2 * M * N * K / us / 1e6:7.1f} TFLOP/s', flush=True)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else None)
