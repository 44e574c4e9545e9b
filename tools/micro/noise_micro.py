"""F (cc_noise_fwd) alone at the bench configuration (V=22000, B=512, C=65536 synthetic cubes):
kernel time by HIP events, and per-phase durations from the probe copy of the kernel (dev tool).
Phases: 0 start -> 1 bits cleared -> 2 cube bits + k -> 3 cut draws -> 4 add draws -> 5 x/y
bitmask rows + count scan -> 6 compaction written."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)
from cubecobrarecommender_amd import _lib as L  # noqa: E402


def build_probe():
    so = os.path.join(ROOT, 'tools', 'micro', 'libnoise_probe.so')
    src = os.path.join(ROOT, 'tools', 'micro', 'noise_probe.hip')
    pkg = os.path.join(ROOT, 'cubecobrarecommender_amd')
    deps = (src, os.path.join(pkg, 'csrc', 'noise.hip'))
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(f) for f in deps):
        subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '-fPIC', '-shared',
                               '-I', os.path.join(ROOT, 'include'), '-I', os.path.join(pkg, 'csrc'), src,
                               '-L', pkg, '-lccrec_hip', '-Wl,-rpath,' + pkg, '-Wl,-Bsymbolic', '-o', so])
    return so


def main():
    so = build_probe()
    if not torch.cuda.is_available():
        return
    from cubecobrarecommender_amd.synthetic import synthetic_cubes, neg_sampler_from_csr
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    from cubecobrarecommender_amd.layout import glorot_flat
    V, d, B = 22000, 256, 512
    indptr, indices = synthetic_cubes(65536, V, seed=20250301, device='cuda')
    ns = neg_sampler_from_csr(indptr, indices, V)
    data = DeviceDataset(csr=(indptr, indices), num_cards=V, neg_sampler=ns, device='cuda')
    tr = Trainer(TrainConfig(V=V, d=d, batch_size=B, dtype='bf16', seed=1234), data,
                 params_flat=glorot_flat(V, d, seed=42), device=torch.device('cuda', 0))
    rng = np.random.default_rng(99)
    tr.set_epoch_permutations(np.stack([rng.permutation(65536) for _ in range(4)]))
    na = tr._noise_args()
    s = L.stream_ptr(None)
    for _ in range(5):
        L.call('cc_noise_fwd', ctypes.byref(na), s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        L.call('cc_noise_fwd', ctypes.byref(na), s)
    e1.record()
    torch.cuda.synchronize()
    print('cc_noise_fwd alone: %.2f us' % (e0.elapsed_time(e1) / 50 * 1e3))
    pl = ctypes.CDLL(so)
    for _ in range(3):
        pl.noise_probe_fwd(ctypes.byref(na), s)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (1024 * 8))()
    pl.noise_probe_read(buf, 1024 * 8)
    t = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8)[:B, :7].astype(np.int64)
    t0 = t[:, 0].min()
    print('block start spread (us): max %.2f' % ((t[:, 0].max() - t0) / 100.0))
    print('block end (us from first start): mean %.2f max %.2f' % ((t[:, 6] - t0).mean() / 100.0, (t[:, 6] - t0).max() / 100.0))
    ph = np.diff(t, axis=1) / 100.0    # wall_clock64: 100 MHz
    for k in range(6):
        print('phase %d->%d: mean %.2f  p50 %.2f  max %.2f us' % (k, k + 1, ph[:, k].mean(), np.median(ph[:, k]), ph[:, k].max()))
    cnt = tr.x_cnt[:B].float()
    print('mean x_cnt %.1f' % cnt.mean().item())


if __name__ == '__main__':
    main()
