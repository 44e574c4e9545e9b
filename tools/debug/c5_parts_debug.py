"""Debug: the fp8 data-parallel step's graph-part path (the first step after a capture: the
captured forward_backward_a / _b replayed around the eager exchange) against the same step run
eagerly, gradient buffer snapshots after each phase (1-rank RCCL group)."""
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
a = _rccl_trainer(shape, reg, True, shard)
e = _rccl_trainer(shape, reg, True, shard)
for t in (a, e):
    for _ in range(2):
        t.step()
    torch.cuda.synchronize()
a.capture()
torch.cuda.synchronize()
snaps = {'a': {}, 'e': {}}


def wrap(name, key, f):
    def g():
        f()
        torch.cuda.synchronize()
        snaps[name][key] = (a if name == 'a' else e).grads.clone().cpu().numpy()
    return g


for name, t, g in (('a', a, a.graphs), ('e', e, None)):
    sh = t._sharded()
    t.noise_ready = False
    sh.step(phase_a=wrap(name, 'A', g[0].replay if g else t.forward_backward_a),
            phase_b=wrap(name, 'B', g[1].replay if g else t.forward_backward_b),
            rest=g[2].replay if g else t.apply_rest,
            adam_fn=lambda lo, n, gs, t=t: t.adam_range(lo, n, gs),
            refresh_fn=lambda lo, hi, t=t: t.refresh_range(lo, hi), after_b=None, hooks=False)
    torch.cuda.synchronize()
    snaps[name]['gfull'] = sh.bucket('biases')['gfull'].cpu().numpy()
lay = a.layout
for key in ('A', 'B'):
    x, y = snaps['a'][key], snaps['e'][key]
    bad = np.nonzero(~(x == y) & ~(np.isnan(x) & np.isnan(y)))[0]
    print(key, 'differing grads elements', bad.size)
    for name, (o, shp) in lay.entries.items():
        n = int(np.prod(shp))
        sel = bad[(bad >= o) & (bad < o + n)]
        if sel.size:
            print('   ', name, sel.size, 'first', int(sel[0] - o), x[sel[0]], y[sel[0]])
    outside = [i for i in bad if not any(o <= i < o + int(np.prod(s)) for o, s in lay.entries.values())]
    print('    outside tensors:', len(outside), outside[:8])
x, y = snaps['a']['gfull'], snaps['e']['gfull']
print('gfull differing', int((x != y).sum()), np.nonzero(x != y)[0][:8])
dist.destroy_process_group()
