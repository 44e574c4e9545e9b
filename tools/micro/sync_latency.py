"""Host-side cost of a bracketed GPU interval: synchronize; t0; one tiny launch (or a graph replay);
synchronize; t1 — with the runtime's default device scheduling or with spin-waiting
(hipSetDeviceFlags(hipDeviceScheduleSpin) before any GPU call).  Dev tool:
    python tools/micro/sync_latency.py [spin]"""
import ctypes
import sys
import time

spin = len(sys.argv) > 1 and sys.argv[1] == 'spin'
if spin:
    hip = ctypes.CDLL('libamdhip64.so')
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))   # hipDeviceScheduleSpin
    print('hipSetDeviceFlags(spin) ->', rc)
import numpy as np
import torch

x = torch.zeros(1 << 20, device='cuda')
for _ in range(20):
    x.add_(1)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    x.add_(1)
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    for _ in range(8):
        x.add_(1)
torch.cuda.synchronize()
for name, fn in (('launch', lambda: x.add_(1)), ('graph8', g.replay)):
    ts = []
    for _ in range(200):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts[20:]) * 1e6
    print(f'{"spin" if spin else "default"} {name}: median {np.median(ts):.1f} us, p10 {np.percentile(ts, 10):.1f}, p90 {np.percentile(ts, 90):.1f}')
