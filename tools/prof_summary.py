"""Render a rocprofv3 kernel_stats.csv as a markdown table (profiles/*_summary.md).

python tools/prof_summary.py STATS_CSV TITLE COMMAND [BENCH_JSON] > profiles/<name>_summary.md
"""
import csv
import json
import sys


def main():
    path, title, cmd = sys.argv[1:4]
    bench = sys.argv[4] if len(sys.argv) > 4 else None
    rows = list(csv.DictReader(open(path)))
    print(f'# {title}\n')
    print(f'Command: `{cmd}`  ')
    print(f'Full table: `{path.split("/")[-1]}` (copied next to this file).\n')
    if bench:
        lines = [l for l in open(bench) if l.startswith('{')]
        if lines:
            b = json.loads(lines[-1])
            r = b.get('roofline', {})
            print(f"Bench (no profiler): {b['value']:.0f} {b['unit']}, {b['ms_per_step'] * 1e3:.1f} us/step; "
                  f"roofline kernel {r.get('kernel')} avg {r.get('avg_ms', 0) * 1e3:.1f} us "
                  f"({r.get('achieved', 0):.0f} {r.get('unit')}, frac {r.get('frac', 0):.3f}).\n")
    print('| kernel | calls | avg us | % of GPU time |')
    print('|---|---|---|---|')
    for r in rows[:30]:
        name = r['Name'].replace('|', '/')[:100]
        print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")


if __name__ == '__main__':
    main()
