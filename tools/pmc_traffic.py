#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes into per-launch HBM traffic for a kernel (MI355X_MICROARCH.md §HBM):
FETCH_SIZE and WRITE_SIZE (KB, from TCC_EA0_RDREQ/WRREQ) are collected in SEPARATE passes; on gfx950
FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

usage: pmc_traffic.py <kernel-substring> <fetch_pass_dir> <write_pass_dir> <out.json> [key]
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kname):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    vals = {}
    for db in glob.glob(os.path.join(d, '**', '*.db'), recursive=True):   # rocprofv3 rocpd output
        import sqlite3
        c = sqlite3.connect(db)
        for disp, name, cn, v in c.execute(
                'select dispatch_id, kernel_name, counter_name, value from counters_collection'):
            if counter in cn and kname in name:
                vals[(db, disp)] = vals.get((db, disp), 0.0) + float(v)
    for f in files:
        for r in csv.DictReader(open(f)):
            if counter not in r.get('Counter_Name', '') or kname not in r.get('Kernel_Name', ''):
                continue
            key = r.get('Dispatch_Id') or r.get('Correlation_Id') or str(len(vals))
            vals[key] = vals.get(key, 0.0) + float(r['Counter_Value'])
    return list(vals.values())


def main():
    kname, dfetch, dwrite, out = sys.argv[1:5]
    key = sys.argv[5] if len(sys.argv) > 5 else kname
    f = per_dispatch(dfetch, 'FETCH_SIZE', kname)
    w = per_dispatch(dwrite, 'WRITE_SIZE', kname)
    if not f or not w:
        print('no samples', len(f), len(w))
        sys.exit(1)
    fetch_b = 2.0 * 1024 * sum(f) / len(f)
    write_b = 1024 * sum(w) / len(w)
    res = json.load(open(out)) if os.path.exists(out) else {}
    res[key] = {'bytes_per_launch': fetch_b + write_b, 'fetch_bytes': fetch_b, 'write_bytes': write_b,
                'dispatches': [len(f), len(w)],
                'method': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; '
                          'FETCH_SIZE x2 (gfx950 16-B/lane read correction), x1024 (KB)'}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res[key]))


if __name__ == '__main__':
    main()
