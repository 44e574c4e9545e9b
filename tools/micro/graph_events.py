"""Can timing events be recorded inside a captured graph on this ROCm build, and what does a
graph boundary cost?  Prints elapsed times of in-graph events and of back-to-back replays."""
import torch

x = torch.randn(64 << 20, device='cuda')
y = torch.empty_like(x)
s = torch.cuda.Stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    y.copy_(x)  # warm
    torch.cuda.synchronize()
    ok = True
    try:
        with torch.cuda.graph(g, stream=s):
            y.copy_(x)
            e0.record()
            y.mul_(2.0)
            e1.record()
            y.add_(1.0)
    except Exception as ex:  # noqa: BLE001
        ok = False
        print('capture with events failed:', repr(ex)[:300])
torch.cuda.synchronize()
if ok:
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    try:
        print('in-graph event elapsed ms:', e0.elapsed_time(e1))
    except Exception as ex:  # noqa: BLE001
        print('elapsed_time failed:', repr(ex)[:300])

# graph boundary cost: N small graphs vs one graph with N kernels
small = [torch.cuda.CUDAGraph() for _ in range(3)]
z = torch.zeros(1024, device='cuda')
with torch.cuda.stream(s):
    for gg in small:
        with torch.cuda.graph(gg, stream=s):
            for _ in range(5):
                z.add_(1.0)
    big = torch.cuda.CUDAGraph()
    with torch.cuda.graph(big, stream=s):
        for _ in range(15):
            z.add_(1.0)
torch.cuda.synchronize()
for name, fn in [('3 graphs x 5 kernels', lambda: [gg.replay() for gg in small]),
                 ('1 graph x 15 kernels', lambda: big.replay())]:
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(name, 'us per iteration:', a.elapsed_time(b) / 200 * 1e3)
