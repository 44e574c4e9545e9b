"""Time cc_dec_bce_dw (fused D1 output layer) alone at the bench shape (dev tool; run under
rocprofv3 --kernel-trace --stats or --pmc)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402

B, V, d = 512, int(os.environ.get('V', '22000')), 256
bf = dict(device='cuda', dtype=torch.bfloat16)
D3 = (torch.randn(B, d, device='cuda') * 0.5).to(torch.bfloat16)
D3t = D3.t().contiguous()
WoT = (torch.randn(V, d, device='cuda') * 0.05).to(torch.bfloat16)
bo = torch.zeros(V, device='cuda')
ybits = torch.randint(-2**31, 2**31 - 1, (B, (V + 31) // 32), device='cuda', dtype=torch.int32)
dZ = torch.empty(B, V, **bf)
gW = torch.empty(d, V, device='cuda')
gb = torch.empty(V, device='cuda')
part = torch.zeros(4096, device='cuda', dtype=torch.float64)
loss = torch.zeros(1, device='cuda', dtype=torch.float64)
tick = torch.zeros(1, device='cuda', dtype=torch.int32)
D3p = D3.view(B // 32, 32, d // 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous()
D3tp = D3t.view(d // 32, 32, B // 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous()
PK = [None, None]
WoD = [None]
Wo = WoT.t().contiguous()


def run():
    L.call('cc_dec_bce_dw', L.ptr(D3), L.ptr(D3t), B, PK[0], PK[1], None if WoD[0] else L.ptr(WoT), WoD[0], L.ptr(bo), B, d, V, L.ptr(ybits),
           L.ptr(dZ), L.ptr(gW), L.ptr(gb), L.ptr(part), L.ptr(loss), 1.0 / (B * V), L.ptr(tick),
           L.stream_ptr())


for pk in (0, 1, 2):
    PK[:] = [L.ptr(D3p), L.ptr(D3tp)] if pk else [None, None]
    WoD[0] = L.ptr(Wo) if pk == 2 else None
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = int(os.environ.get('N', '50'))
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f'dec_bce_dw packed={pk} {e0.elapsed_time(e1) / n * 1000:.1f} us (dbg={os.environ.get("CCREC_DECOUT_DBG", "0")}, V={V})')
