"""Debug: the fp8 data-parallel step (1-rank RCCL group) replayed from graphs against the same
trainer run eagerly, compared after every step for N steps; every capture() is followed by one
graph-part step (the first step after a capture), so argv recap=K re-captures every K steps to
exercise it repeatedly.  Reports the first step and tensor elements that differ."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
torch.cuda.set_device(0)
dist.init_process_group('nccl', store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device('cuda', 0))
from tests.test_gpu_dp import _rccl_trainer  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else 'c5'
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
recap = int(sys.argv[3]) if len(sys.argv) > 3 else 4
a = _rccl_trainer(shape, 0.1, True, True)
e = _rccl_trainer(shape, 0.1, True, True)
lay = a.layout
for step in range(nsteps):
    if step % recap == 1:
        a.capture()
    path = 'graph' if (a.g_dp is not None and a.noise_ready) else ('parts' if a.graphs is not None else 'eager')
    for t in (a, e):
        t.step()
    torch.cuda.synchronize()
    bad_any = False
    for what in ('params', 'm', 'v', 'shadow', 'grads'):
        x, y = getattr(a, what).float().cpu().numpy(), getattr(e, what).float().cpu().numpy()
        bad = np.nonzero(~(x == y) & ~(np.isnan(x) & np.isnan(y)))[0]
        if bad.size:
            bad_any = True
            names = {}
            for nm, (o, shp) in lay.entries.items():
                sel = bad[(bad >= o) & (bad < o + int(np.prod(shp)))]
                if sel.size:
                    names[nm] = (int(sel.size), [int(i - o) for i in sel[:6]], [float(x[i]) for i in sel[:3]],
                                 [float(y[i]) for i in sel[:3]])
            print(f'step {step} ({path}) {what}: {bad.size} differ {names}', flush=True)
    if not bad_any:
        print(f'step {step} ({path}) identical', flush=True)
    else:   # continue from identical states
        for what in ('params', 'm', 'v', 'shadow'):
            getattr(a, what).copy_(getattr(e, what))
dist.destroy_process_group()
