"""Time cc_embed_grad_mfma alone at the bench shape (V=22000, d=256, R=512; dev tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402

V, d, R = 22000, int(os.environ.get('D', '256')), 512
rng = np.random.default_rng(0)
p = 437.0 / V
X = rng.random((R, V)) < p
xt = np.zeros((V, R // 32), np.uint32)
rr, cc = np.nonzero(X)
np.bitwise_or.at(xt, (cc, rr // 32), (np.uint32(1) << (rr % 32).astype(np.uint32)))
xt0 = torch.from_numpy(xt.view(np.int32)).cuda()
xtd = xt0.clone()
gT = torch.randn(d, R, device='cuda').to(torch.bfloat16)
grad = torch.empty(V, d, device='cuda')
bg = torch.empty(d, device='cuda')
n = 50
ts = []
for i in range(n + 3):
    xtd.copy_(xt0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    L.call('cc_embed_grad_mfma', L.ptr(gT), V, d, R, R, L.ptr(xtd), L.ptr(grad), L.ptr(bg), L.stream_ptr())
    e1.record()
    ts.append((e0, e1))
torch.cuda.synchronize()
t = np.median([a.elapsed_time(b) for a, b in ts[3:]]) * 1000
print(f'embed_grad_mfma d={d} NC={os.environ.get("CCREC_EG_NC", "128")}: {t:.1f} us')
