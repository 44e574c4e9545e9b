"""Print the top kernels of a prof_collect stats CSV per step: calls/step, us/call, us/step.
usage: python tools/kstat.py STATS.csv STEPS [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
out = []
for r in rows:
    calls = int(r['Calls'])
    if calls < steps * 0.9:   # once-per-run kernels (setup, recommend) are not per step
        continue
    out.append((float(r['TotalDurationNs']) / 1e3 / calls * round(calls / steps), calls / steps,
                float(r['AverageNs']) / 1e3, r['Name']))
out.sort(reverse=True)
tot = sum(o[0] for o in out)
for per_step, cps, avg, name in out[:n]:
    print(f'{per_step:8.1f} us/step {cps:5.1f}x {avg:8.1f} us  {name[:90]}')
print(f'{tot:8.1f} us/step summed over per-step kernels')
