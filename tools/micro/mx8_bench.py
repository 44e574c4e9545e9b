"""Time config 5's MX-FP8 decoder GEMM shapes through cc_gemm (dev tool): the generic NT kernel at
d = 1024, |V| = 22,000, B = 512, with and without its epilogues, next to the bf16 kernel on the same
shapes.  Prints torch-event averages per variant (run under rocprofv3 --stats for kernel times)."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402

B, V, d = 512, 22000, 1024
Vp = (V + 127) // 128 * 128
dev = 'cuda'
u8 = dict(device=dev, dtype=torch.uint8)
bf = dict(device=dev, dtype=torch.bfloat16)


def codes(r, c):   # finite e4m3 codes (no NaN patterns)
    return torch.randint(0, 0x70, (r, c), **u8)


def scales(r, c):
    return torch.full((r, c // 32), 120, **u8)


D3q, D3qs = codes(B, d), scales(B, d)
D3tq, D3tqs = codes(d, B), scales(d, B)
WoT8, WoT8s = codes(V, d), scales(V, d)
Wo8, Wo8s = codes(d, Vp), scales(d, Vp)
dZq, dZqs = codes(B, Vp), scales(B, Vp)
dZtq, dZtqs = codes(V, B), scales(V, B)
D3 = torch.randn(B, d, **bf)
WoT = torch.randn(V, d, **bf) * 0.05
bias = torch.zeros(V, device=dev)
gbias = torch.zeros(V, device=dev)
ybits = torch.randint(0, 2**31 - 1, (B, (V + 31) // 32), device=dev, dtype=torch.int32)
part = torch.zeros(8192, device=dev, dtype=torch.float64)
Cb = torch.empty(B, V, **bf)
Ct = torch.empty(V, B, **bf)
Z2 = torch.empty(B, V, device=dev)
gW = torch.empty(d, V, device=dev)
split = torch.empty(64 * B * d, device=dev)


def args(M, N, K, A, lda, Bp, ldb, epi, mx=True, sa=None, sb=None, **kw):
    g = L.GemmArgs()
    g.dtype, g.ta, g.tb, g.epilogue = (L.CC_MX8 if mx else L.CC_BF16), 0, 1, epi
    g.M, g.N, g.K, g.lda, g.ldb, g.ldc, g.splits, g.relu = M, N, K, lda, ldb, kw.get('ldc', N), kw.get('splits', 1), 0
    g.A, g.B = A.data_ptr(), Bp.data_ptr()
    g.a_scale = sa.data_ptr() if sa is not None else None
    g.b_scale = sb.data_ptr() if sb is not None else None
    for k in ('bias', 'C', 'Cf', 'y_bits', 'loss_partials', 'colsum', 'Ct'):
        v = kw.get(k)
        setattr(g, k, v.data_ptr() if v is not None else None)
    g.scale = 1.0 / (B * V)
    g.ldct = kw.get('ldct', 0)
    return g


def gemm(*a, **kw):
    L.call('cc_gemm', C.byref(args(*a, **kw)), L.stream_ptr())


def pair(ga, gb_):
    L.call('cc_gemm_pair', C.byref(ga), C.byref(gb_), L.stream_ptr())


def main(only=None):
    S = 16
    variants = {
        'mx8 logits+bce+C+Ct': lambda: gemm(B, V, d, D3q, d, WoT8, d, L.CC_EPI_BCE, sa=D3qs, sb=WoT8s, bias=bias,
                                            C=Cb, y_bits=ybits, loss_partials=part, Ct=Ct, ldct=B),
        'mx8 bce_q': lambda: L.call('cc_gemm_mx8_bce_q', C.byref(args(
            B, V, d, D3q, d, WoT8, d, L.CC_EPI_BCE, sa=D3qs, sb=WoT8s, bias=bias, y_bits=ybits, loss_partials=part)),
            L.ptr(dZq), Vp, L.ptr(dZqs), L.ptr(dZtq), B, L.ptr(dZtqs), L.ptr(gbias), L.stream_ptr()),
        'mx8 logits compute': lambda: gemm(B, V, d, D3q, d, WoT8, d, L.CC_EPI_STORE, sa=D3qs, sb=WoT8s),
        'mx8 reg logits Cf': lambda: gemm(B, V, d, D3q, d, WoT8, d, L.CC_EPI_STORE, sa=D3qs, sb=WoT8s, bias=bias, Cf=Z2),
        'mx8 dX splitk16': lambda: gemm(B, d, Vp, dZq, Vp, Wo8, Vp, L.CC_EPI_SPLITK, sa=dZqs, sb=Wo8s, Cf=split, splits=S),
        'mx8 dW Cf': lambda: gemm(d, V, B, D3tq, B, dZtq, B, L.CC_EPI_STORE, sa=D3tqs, sb=dZtqs, Cf=gW),
        'mx8 dW compute': lambda: gemm(d, V, B, D3tq, B, dZtq, B, L.CC_EPI_STORE, sa=D3tqs, sb=dZtqs),
        'mx8 pair dX+dW': lambda: pair(args(B, d, Vp, dZq, Vp, Wo8, Vp, L.CC_EPI_SPLITK, sa=dZqs, sb=Wo8s, Cf=split, splits=S),
                                       args(d, V, B, D3tq, B, dZtq, B, L.CC_EPI_STORE, sa=D3tqs, sb=dZtqs, Cf=gW)),
        'bf16 logits compute': lambda: gemm(B, V, d, D3, d, WoT, d, L.CC_EPI_STORE, mx=False),
    }
    for name, fn in variants.items():
        if only and name != only:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f'{name:22s} {e0.elapsed_time(e1) / 30 * 1000:8.1f} us', flush=True)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else None)
