"""dX = dZ . Wo^T at the bench shape (B=512, V=22000, d=256): our split-K cc_gemm + reduce vs the
library GEMM (torch.mm -> hipBLASLt/rocBLAS), events over back-to-back launches (dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench as G  # noqa: E402


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


dZ, Wo = G.dZ, G.Wo
out = torch.empty(G.B, G.d, device='cuda', dtype=torch.bfloat16)


def ours(splits):
    G.gemm(G.B, G.d, G.V, dZ, G.V, Wo, G.V, G.L.CC_EPI_SPLITK, Cf=G.split, splits=splits)
    G.L.call('cc_splitk_reduce', G.L.CC_BF16, G.L.ptr(G.split), splits, G.B, G.d, None, G.L.ptr(out), None,
             None, None, G.L.stream_ptr())


for s in (16, 32, 64):
    print('ours splitk%d + reduce  %.1f us' % (s, timeit(lambda: ours(s))))
print('torch.mm bf16 out       %.1f us' % timeit(lambda: torch.mm(dZ, Wo.t(), out=out)))
ref = dZ.float() @ Wo.float().t()
torch.mm(dZ, Wo.t(), out=out)
print('max rel err torch bf16', ((out.float() - ref).abs().max() / ref.abs().max()).item())
