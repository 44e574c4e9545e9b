"""Debug: the fp8 data-parallel step's graph-part path (the first step after a capture: the
captured forward_backward_a / _b replayed around the eager exchange) against the same step run
eagerly — gradient snapshots after each phase, the biases bucket's all-reduced gradient, and the
parameters / moments after the step (1-rank RCCL group).  argv: shape reg shard after_b(0/1)."""
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
reg = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
shard = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
use_after = bool(int(sys.argv[4])) if len(sys.argv) > 4 else True
a = _rccl_trainer(shape, reg, True, shard)
e = _rccl_trainer(shape, reg, True, shard)
for t in (a, e):
    for _ in range(2):
        t.step()
    torch.cuda.synchronize()
a.capture()
torch.cuda.synchronize()
snaps = {'a': {}, 'e': {}}


def wrap(name, key, t, f):
    def g():
        f()
        torch.cuda.synchronize()
        snaps[name][key] = t.grads.clone().cpu().numpy()
    return g


for name, t, g in (('a', a, a.graphs), ('e', e, None)):
    sh = t._sharded()
    t.noise_ready = False
    sh.step(phase_a=wrap(name, 'A', t, g[0].replay if g else t.forward_backward_a),
            phase_b=wrap(name, 'B', t, g[1].replay if g else t.forward_backward_b),
            rest=g[2].replay if g else t.apply_rest,
            adam_fn=lambda lo, n, gs, t=t: t.adam_range(lo, n, gs),
            refresh_fn=lambda lo, hi, t=t: t.refresh_range(lo, hi),
            after_b=t.noise_next if use_after else None, hooks=False)
    t.noise_ready = use_after and t.prefetch_dp
    torch.cuda.synchronize()
    snaps[name]['gfull'] = sh.bucket('biases')['gfull'].cpu().numpy()
    for what in ('params', 'm', 'v', 'shadow'):
        snaps[name][what] = getattr(t, what).float().cpu().numpy()
lay = a.layout
for key in ('B', 'params', 'm', 'v', 'shadow'):
    x, y = snaps['a'][key], snaps['e'][key]
    bad = np.nonzero(~(x == y) & ~(np.isnan(x) & np.isnan(y)))[0]
    print(key, 'differing elements', bad.size)
    for nm, (o, shp) in lay.entries.items():
        n = int(np.prod(shp))
        sel = bad[(bad >= o) & (bad < o + n)]
        if sel.size:
            print('   ', nm, sel.size, 'first', int(sel[0] - o), x[sel[0]], y[sel[0]])
x, y = snaps['a']['gfull'], snaps['e']['gfull']
print('gfull differing', int((x != y).sum()), np.nonzero(x != y)[0][:8])


def compare(tag):
    torch.cuda.synchronize()
    for what in ('params', 'm', 'v', 'shadow'):
        x, y = getattr(a, what).float().cpu().numpy(), getattr(e, what).float().cpu().numpy()
        bad = np.nonzero(~(x == y) & ~(np.isnan(x) & np.isnan(y)))[0]
        names = {}
        for nm, (o, shp) in lay.entries.items():
            sel = bad[(bad >= o) & (bad < o + int(np.prod(shp)))]
            if sel.size:
                names[nm] = (int(sel.size), [int(i - o) for i in sel[:4]], [float(x[i]) for i in sel[:2]],
                             [float(y[i]) for i in sel[:2]])
        print(tag, what, 'differing', bad.size, names)


# the same two trainers through Trainer.step (a: the whole-step graph replay; e: eager with hooks)
for k in range(3):
    for t in (a, e):
        t.step()
    compare(f'graph step {k}')
# the whole-step graph captured without the early first-bucket hooks
sh = a._sharded()
orig = sh.step
sh.step = lambda *args, **kw: orig(*args, **{**kw, 'hooks': False})
a._capture_dp()
sh.step = orig
a.noise_ready = True
e2 = e
for k in range(2):
    for t in (a, e):
        t.step()
    compare(f'no-hook graph step {k}')
dist.destroy_process_group()
