"""cc_gemm_dx_splitk + cc_splitk_reduce at the bench shape (M=512, N=256, K=22000) for several
split counts, both tile shapes (128x128; 128x256 via CCREC_DX_WIDE_MIN set in the environment
before the library loads) — events over back-to-back launches (dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402

M, N, K = 512, 256, 22000
dZ = (torch.randn(M, K, device='cuda') * 0.01).to(torch.bfloat16)
Wo = (torch.randn(N, K, device='cuda') * 0.05).to(torch.bfloat16)
D3 = torch.randn(M, N, device='cuda').to(torch.bfloat16)
gD3 = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
part = torch.empty(64 * M * N, device='cuda')
s = L.stream_ptr()


def timeit(fn, n=100):
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


for S in [int(x) for x in os.environ.get('SPLITS', '8 16 24 32 48 64').split()]:
    dx = lambda: L.call('cc_gemm_dx_splitk', L.ptr(dZ), K, L.ptr(Wo), K, M, N, K, S, L.ptr(part), s)
    red = lambda: L.call('cc_splitk_reduce', L.CC_BF16, L.ptr(part), S, M, N, L.ptr(D3), L.ptr(gD3),
                         None, None, None, s)
    both = lambda: (dx(), red())
    print('wide_min=%s S=%d: dx %.1f  reduce %.1f  both %.1f us' % (os.environ.get('CCREC_DX_WIDE_MIN', '4096'), S,
                                                                  timeit(dx), timeit(red), timeit(both)))
ref = (dZ.float() @ Wo.float().t())
ref = torch.where(D3.float() > 0, ref, torch.zeros_like(ref))
print('max abs err', (gD3.float() - ref).abs().max().item())
