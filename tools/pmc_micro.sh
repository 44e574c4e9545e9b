#!/bin/bash
# SQ counter passes (one run each, 60 s kill) over a micro-benchmark, per kernel averages.
# usage: bash tools/pmc_micro.sh TAG "counters pass 1" "counters pass 2" ... -- script.py [args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
passes=()
while [ "$1" != "--" ]; do passes+=("$1"); shift; done
shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for c in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d "$O/pmc$i" -o run -- python3 "$R/$@" > "$O/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/pmc$i.log"; exit 1; }
done
python3 - "$O" <<'PY'
import glob, os, sqlite3, sys
o = sys.argv[1]
agg = {}
for db in glob.glob(os.path.join(o, 'pmc*', '**', '*.db'), recursive=True):
    c = sqlite3.connect(db)
    try:
        rows = c.execute('select kernel_name, counter_name, value from counters_collection').fetchall()
    except Exception as e:
        print('db', db, e); continue
    for k, cn, v in rows:
        a = agg.setdefault((k[:60], cn), [0, 0.0])
        a[0] += 1; a[1] += float(v)
for (k, cn), (n, s) in sorted(agg.items()):
    if any(x in k for x in ('kl_', 'dec_', 'gemm', 'tower', 'embed', 'gather', 'adam')):
        print(f'{k:60s} {cn:28s} {s / n:14.1f}  (n={n})')
PY
