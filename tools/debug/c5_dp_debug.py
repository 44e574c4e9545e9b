"""Debug: the fp8 (config 5 class) step, tensor by tensor, after each step (gradients after step 0,
parameters / moments after each).  Trainers: 'dp' = the data-parallel step over a 1-rank RCCL group,
'one' = the one-process step (both captured at step 2), 'bceq0' = 'one' without the BCE product's
MX-FP8 epilogue, all checked against 'eager' (one-process, never captured)."""
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
tr = {'eager': _rccl_trainer(shape, reg, False, False),
      'one': _rccl_trainer(shape, reg, False, False),
      'bceq0': _rccl_trainer(shape, reg, False, False, mx8_bce_q=False),
      'dp': _rccl_trainer(shape, reg, True, True)}
for step in range(6):
    if step == 2:
        for k in ('one', 'bceq0', 'dp'):
            tr[k].capture()
    for k, t in tr.items():
        t.step()
        t.flush()
        torch.cuda.synchronize()
    print('step', step, 'losses', {k: t.losses()['loss'] for k, t in tr.items()})
    ref = tr['eager']
    for name in ('one', 'bceq0', 'dp'):
        a = tr[name]
        for what in ('grads', 'params', 'm', 'v'):
            if what == 'grads' and step >= 2:
                continue
            ua = a.std_layout.unpack(a.standard(getattr(a, what)))
            ub = ref.std_layout.unpack(ref.standard(getattr(ref, what)))
            bad = []
            for k in ua:
                x, y = ua[k].astype(np.float64), ub[k].astype(np.float64)
                nx, ny = np.isnan(x).sum(), np.isnan(y).sum()
                e = np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30)
                if nx or ny or e > 1e-6:
                    i = int(np.argmax(np.abs(x - y).ravel()))
                    bad.append((k, int(nx), int(ny), float(e), float(np.abs(x).max()), float(np.abs(y).max()), i))
            print(' ', name, what, 'mismatches:', bad if bad else 'none')
dist.destroy_process_group()
