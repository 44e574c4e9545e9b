"""Debug: the fp8 (config 5 class) data-parallel step over a 1-rank RCCL group vs the one-process
step, tensor by tensor (gradients after step 0, parameters / moments after each step)."""
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
b = _rccl_trainer(shape, reg, False, False)
for step in range(3):
    for t in (a, b):
        if t is a:
            t._dp_call(None)
        else:
            t.forward_backward()
            t.apply()
        torch.cuda.synchronize()
    print('step', step, 'losses', a.losses(), b.losses())
    for what in ('grads', 'params', 'm', 'v'):
        ua = a.layout.unpack(a.standard(getattr(a, what)))
        ub = b.layout.unpack(b.standard(getattr(b, what)))
        bad = []
        for k in ua:
            x, y = ua[k].astype(np.float64), ub[k].astype(np.float64)
            nx, ny = np.isnan(x).sum(), np.isnan(y).sum()
            e = np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30)
            if nx or ny or e > 1e-6:
                bad.append((k, int(nx), int(ny), float(e), float(np.abs(x).max()), float(np.abs(y).max())))
        print(' ', what, 'mismatches:', bad if bad else 'none')
dist.destroy_process_group()
