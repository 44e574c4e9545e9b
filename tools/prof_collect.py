#!/usr/bin/env python3
"""Reduce one rocprofv3 output directory (rocpd sqlite databases) to small files on the GPU box, so
that gpurun_out/ stays well under the copy-back limit, then delete the raw databases.

  stats DIR OUT.csv    kernel statistics (Name, Calls, TotalDurationNs, AverageNs, Percentage,
                       MinNs, MaxNs), sorted by total time
  pmc   DIR OUT.json   per-kernel average (over dispatches) of every collected counter, plus the
                       dispatch count and the kernels' average duration when the db holds it
  timeline DIR OUT.csv the last 80 kernel dispatches in start order: name, start and duration (ns)
                       and the idle gap before each (launch boundaries inside a graph replay)
"""
import csv
import glob
import json
import os
import shutil
import sqlite3
import sys


def dbs_of(d):
    return glob.glob(os.path.join(d, '**', '*.db'), recursive=True)


def stats(d, out):
    agg = {}
    for db in dbs_of(d):
        c = sqlite3.connect(db)
        for name, dur in c.execute('select name, duration from kernels'):
            a = agg.setdefault(name, [0, 0.0, float('inf'), 0.0])
            a[0] += 1
            a[1] += dur
            a[2] = min(a[2], dur)
            a[3] = max(a[3], dur)
    if not agg:
        raise SystemExit(f'no kernels in {d}')
    tot = sum(a[1] for a in agg.values()) or 1.0
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs'])
        for name, (n, t, lo, hi) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, n, int(t), t / n, 100.0 * t / tot, int(lo), int(hi)])


def pmc(d, out):
    per = {}
    for db in dbs_of(d):
        c = sqlite3.connect(db)
        rows = c.execute('select dispatch_id, kernel_name, counter_name, value from counters_collection').fetchall()
        for disp, k, cn, v in rows:
            e = per.setdefault(k, {}).setdefault(cn, {})
            e[(db, disp)] = e.get((db, disp), 0.0) + float(v)   # sum over dimensions per dispatch
    if not per:
        raise SystemExit(f'no counters in {d}')
    res = {}
    for k, cs in per.items():
        r = {}
        for cn, vals in cs.items():
            r[cn] = sum(vals.values()) / len(vals)
            r['dispatches'] = len(vals)
        res[k] = r
    json.dump(res, open(out, 'w'), indent=1, sort_keys=True)


def timeline(d, out, last=80):
    rows = []
    for db in dbs_of(d):
        c = sqlite3.connect(db)
        cur = c.execute('select * from kernels limit 1')
        cols = [x[0] for x in cur.description]
        st = next(x for x in cols if x in ('start', 'start_ns', 'begin', 'start_timestamp'))
        en = next(x for x in cols if x in ('end', 'end_ns', 'stop', 'end_timestamp'))
        rows += c.execute(f'select name, {st}, {en} from kernels').fetchall()
    rows.sort(key=lambda r: r[1])
    rows = rows[-last:]
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Name', 'StartNs', 'DurationNs', 'GapBeforeNs'])
        prev = None
        for name, s0, e0 in rows:
            w.writerow([name[:100], s0 - rows[0][1], e0 - s0, (s0 - prev) if prev is not None else 0])
            prev = e0


def main():
    mode, d, out = sys.argv[1:4]
    {'stats': stats, 'pmc': pmc, 'timeline': timeline}[mode](d, out)
    shutil.rmtree(d, ignore_errors=True)


if __name__ == '__main__':
    main()
