"""First vs later replays of a freshly captured hipGraph, with and without hipGraphUpload before the
first (dev tool): python tools/micro/graph_first_replay.py"""
import ctypes
import time

import numpy as np
import torch

hip = ctypes.CDLL('libamdhip64.so')
x = torch.zeros(1 << 22, device='cuda')
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        x.add_(1)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


for upload in (False, True, False, True):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(72):
            x.add_(1)
    torch.cuda.synchronize()
    if upload:
        rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
    t = [timed(g.replay) for _ in range(6)]
    print(f'upload={upload}: replays (us) ' + ' '.join(f'{v:.0f}' for v in t))
