#!/bin/bash
# rocprofv3 kernel stats of a micro-benchmark: bash tools/prof_micro.sh TAG script.py [args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 "$R/$@" > "$O/prof.log" 2>&1
rc=$?
grep -v "^[WIE]2026" "$O/prof.log" | tail -3
python3 "$R/tools/rocpd_stats.py" "$O/prof" "$O/stats.csv" && python3 - "$O/stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}")
PY
exit $rc
