#!/usr/bin/env python3
"""Kernel statistics of a rocprofv3 rocpd database (its default output format) as the
kernel_stats.csv columns rocprofv3 --stats writes (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs), sorted by total time.

usage: rocpd_stats.py <dir-or-db> <out.csv>
"""
import csv
import glob
import os
import sqlite3
import sys


def main():
    src, out = sys.argv[1:3]
    dbs = [src] if src.endswith('.db') else glob.glob(os.path.join(src, '**', '*.db'), recursive=True)
    agg = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, dur in c.execute('select name, duration from kernels'):
            a = agg.setdefault(name, [0, 0.0, float('inf'), 0.0])
            a[0] += 1
            a[1] += dur
            a[2] = min(a[2], dur)
            a[3] = max(a[3], dur)
    tot = sum(a[1] for a in agg.values()) or 1.0
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs'])
        for name, (n, t, lo, hi) in rows:
            w.writerow([name, n, int(t), t / n, 100.0 * t / tot, int(lo), int(hi)])


if __name__ == '__main__':
    main()
