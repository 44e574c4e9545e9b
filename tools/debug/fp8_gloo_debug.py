"""Debug: configs[4]'s data-parallel fp8 step on two gloo ranks sharing the GPU (the failing
tests/test_gpu_dp.py::test_fp8_dp_step_matches_single_process_and_oracle shape): the same two-rank
run with and without capture(), rank 0's parameters / moments / gradients compared after every step,
differing elements reported per tensor."""
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
STEPS = 3


def worker(rank, port, graphs, out, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE='2',
                      LOCAL_RANK='0', HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=2)
        from tests.test_gpu_dp import FP8_DP, _fp8_trainer
        tr, _ = _fp8_trainer(rank, 2, FP8_DP['B'], False)
        if graphs:
            tr.capture()
        for s in range(STEPS):
            tr.step()
            torch.cuda.synchronize()
            if rank == 0:
                np.savez(f'{out}_{s}.npz', params=tr.params.cpu().numpy(), m=tr.m.cpu().numpy(),
                         grads=tr.grads.cpu().numpy(), shadow=tr.shadow.float().cpu().numpy())
        q.put((rank, 'ok'))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e)))
        raise


def run(graphs, out, port):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, graphs, out, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in ps:
        print(q.get(timeout=300), flush=True)
    for p in ps:
        p.join(60)


if __name__ == '__main__':
    from cubecobrarecommender_amd.layout import Layout
    base = os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'gpurun_out', 'fp8dbg')
    os.makedirs(base, exist_ok=True)
    run(True, base + '/g', 29811)
    run(False, base + '/e', 29812)
    from tests.test_gpu_dp import FP8_DP
    lay = Layout(FP8_DP['V'], FP8_DP['d'], align=128, group_biases=True)
    for s in range(STEPS):
        a, b = np.load(f'{base}/g_{s}.npz'), np.load(f'{base}/e_{s}.npz')
        for what in ('grads', 'params', 'm', 'shadow'):
            x, y = a[what], b[what]
            bad = np.nonzero(~(x == y) & ~(np.isnan(x) & np.isnan(y)))[0]
            names = {}
            for nm, (o, shp) in lay.entries.items():
                sel = bad[(bad >= o) & (bad < o + int(np.prod(shp)))]
                if sel.size:
                    names[nm] = (int(sel.size), [int(i - o) for i in sel[:5]], [float(x[i]) for i in sel[:2]],
                                 [float(y[i]) for i in sel[:2]])
            outside = int(bad.size - sum(v[0] for v in names.values()))
            print(f'step {s} {what}: {bad.size} differ (outside tensors {outside}) {names}', flush=True)
    for f in os.listdir(base):
        os.remove(os.path.join(base, f))
