"""Idle time between two steps of the replayed multi-step graph WITHOUT a profiler (dev tool):
runs bench.py in-process against the probe build of the library (CCREC_LIB=.../libccrec_hip_ts.so,
built with CCREC_BUILD_TAG=ts CCREC_EXTRA_FLAGS=-DCCREC_TS_PROBE=1), then reads the wall-clock
stamps csrc/ts_probe.hpp leaves per step: the Adam + next-F launch's first block start and last
block end, and the next step's E1 gather's first block start.  Prints the distribution of the
boundary gap (gather start - Adam end) and of the Adam launch's duration, in us.

(The probe macros were removed from the product kernels after the measurement; rebuild the probe
library from commit c87345e.)

usage: CCREC_LIB=$PWD/cubecobrarecommender_amd/libccrec_hip_ts.so python tools/micro/gap_probe.py [bench args]
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', '..'))


def main():
    import bench
    sys.argv = ['bench.py', '--no-cpu-baseline', '--no-recommend'] + sys.argv[1:]
    bench.main()
    from cubecobrarecommender_amd import _lib
    L = _lib.lib()
    arr = C.c_ulonglong * 1024
    nf, nl, ef, el = arr(), arr(), arr(), arr()
    assert L.cc_ts_dump_noise(nf, nl) == 0 and L.cc_ts_dump_embed(ef, el) == 0
    nf, nl, ef = (np.array(a[:], dtype=np.int64) for a in (nf, nl, ef))
    ok = (nl > 0) & (ef > 0) & (nf > 0) & (ef > nl)
    gap = (ef - nl)[ok] / 100.0          # s_memrealtime: 100 MHz
    dur = (nl - nf)[ok] / 100.0
    gap = gap[gap < 1000]                 # steps separated by host work (eager / capture) dropped
    print(f'steps with stamps: {int(ok.sum())}; boundary gaps < 1 ms: {gap.size}', flush=True)
    for name, x in (('gap Adam end -> next gather start', gap), ('Adam + F launch duration', dur)):
        q = np.percentile(x, [0, 10, 25, 50, 75, 90, 100])
        print(f'{name:36s} ' + ' '.join(f'{v:7.2f}' for v in q) + '  (min p10 p25 p50 p75 p90 max, us)')
    h, e = np.histogram(gap, bins=[0, 1, 2, 4, 6, 8, 10, 12, 16, 32, 1000])
    print('gap histogram:', {f'{e[i]:g}-{e[i + 1]:g}': int(h[i]) for i in range(len(h))})


if __name__ == '__main__':
    main()
