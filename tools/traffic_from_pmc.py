#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from the reduced PMC passes (tools/prof_collect.py pmc
outputs of separate FETCH_SIZE and WRITE_SIZE runs): bytes = 2 x FETCH_SIZE x 1024 (gfx950: FETCH_SIZE
counts half the bytes of 16-B/lane streaming reads; KB) + WRITE_SIZE x 1024 (MI355X_MICROARCH.md §HBM).
The x2 holds for these kernels' reads: request-size-resolved counters show every TCC_EA0_RDREQ a
128-B request (TCC_EA0_RDREQ_32B = 0, TCC_BUBBLE ~0), and a contiguous 16-B/lane read of a known
11.26 MB gives RDREQ x 128 B = its bytes (tools/micro/d1_fetch_cal.hip, profiles/r06o_d1cal_*.json).

usage: traffic_from_pmc.py <fetch.json> <write.json> <out.json> <kernel-substring>:<key> [...]
"""
import json
import sys


def pick(d, sub):
    ks = [k for k in d if sub in k]
    if not ks:
        raise SystemExit(f'no kernel matching {sub!r}')
    return ks[0], d[ks[0]]


def main():
    fj, wj, out = sys.argv[1:4]
    F, W = json.load(open(fj)), json.load(open(wj))
    res = {}
    for spec in sys.argv[4:]:
        sub, key = spec.split(':')
        kn, f = pick(F, sub)
        _, w = pick(W, sub)
        fetch = 2.0 * 1024.0 * float(f['FETCH_SIZE'])
        write = 1024.0 * float(w['WRITE_SIZE'])
        res[key] = {'bytes_per_launch': fetch + write, 'fetch_bytes': fetch, 'write_bytes': write,
                    'kernel': kn, 'dispatches': f.get('dispatches'),
                    'method': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes '
                              '(tools/gpu_run.sh pmc steps); FETCH_SIZE x2 (every TCC_EA0_RDREQ a 128-B request, '
                              'tallied at 64 B: calibrated in tools/micro/d1_fetch_cal.hip), x1024 (KB); '
                              'per-dispatch averages'}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
