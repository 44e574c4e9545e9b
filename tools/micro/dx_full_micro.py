"""Full-mode decoder_for_reg dX product (dD3 = dZ . Wo^T at M = 22,016 identity rows, K = |V| = 22,000,
N = d = 256, bf16): the library GEMM (torch.mm -> hipBLASLt) vs cc_gemm_dx_splitk at several split
counts (dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402


def t(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    M, K, N = 22016, 22000, 256
    A = (torch.randn(M, K, device='cuda') * 0.01).to(torch.bfloat16)
    Bm = (torch.randn(N, K, device='cuda') * 0.05).to(torch.bfloat16)
    print('torch.mm bf16 out: %.1f us' % t(lambda: torch.mm(A, Bm.t())), flush=True)
    try:
        print('torch.mm fp32 out: %.1f us' % t(lambda: torch.mm(A, Bm.t(), out_dtype=torch.float32)), flush=True)
    except Exception as e:  # noqa: BLE001
        print('no out_dtype:', e)
    for sp in (1, 2, 4):
        P = torch.zeros(sp, M, N, device='cuda')
        s = L.stream_ptr()
        us = t(lambda: L.call('cc_gemm_dx_splitk', L.ptr(A), K, L.ptr(Bm), K, M, N, K, sp, L.ptr(P), s))
        print('cc_gemm_dx_splitk splits %d: %.1f us' % (sp, us), flush=True)


if __name__ == '__main__':
    main()
