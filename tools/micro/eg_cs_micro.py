"""W1-gradient kernels in isolation (dev tool): cc_embed_grad_packed (row tiles, B from L2) vs
cc_embed_grad_cs (column slices, B staged in LDS) at the bench shapes; run under rocprofv3."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402


def main():
    V, d = 22000, 256
    for R in (512, 1024):
        RP = (R + 63) // 64 * 64
        rng = np.random.default_rng(R)
        X = rng.random((R, V)) < 0.02
        xt = np.zeros((V, (R + 31) // 32), np.uint32)
        rr, cc = np.nonzero(X)
        np.bitwise_or.at(xt, (cc, rr // 32), (np.uint32(1) << (rr % 32).astype(np.uint32)))
        xt0 = torch.from_numpy(xt.view(np.int32)).cuda()
        g = (torch.randn(RP, d, device='cuda') * 0.1).to(torch.bfloat16)
        gP = g.view(RP // 16, 2, 8, d // 32, 32).permute(3, 0, 1, 4, 2).contiguous()
        grad = torch.zeros(V, d, device='cuda')
        bg = torch.zeros(d, device='cuda')
        tickets = torch.zeros(int(L.lib().cc_embed_grad_cs_tickets(V, d, R)), device='cuda', dtype=torch.int32)
        xtd = xt0.clone()
        s = L.stream_ptr()
        for rep in range(30):
            xtd.copy_(xt0)
            L.call('cc_embed_grad_packed', L.ptr(gP), V, d, R, RP, L.ptr(xtd), L.ptr(grad), L.ptr(bg), s)
            xtd.copy_(xt0)
            L.call('cc_embed_grad_cs', L.ptr(gP), 1, V, d, R, RP, L.ptr(xtd), L.ptr(grad), L.ptr(bg), L.ptr(tickets), s)
        torch.cuda.synchronize()
        print('R', R, 'done', flush=True)


if __name__ == '__main__':
    main()
