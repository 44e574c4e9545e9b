#!/bin/bash
# BCE step: kernel stats + the last dispatches' timeline (gaps between the graph's kernels)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t9; mkdir -p $O
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-recommend > $R/$O/prof.log 2>&1 || { tail -5 $R/$O/prof.log; exit 1; }
python3 $R/tools/prof_collect.py timeline $R/$O/prof $R/$O/timeline.csv && python3 - <<PY
import csv
r=list(csv.DictReader(open('$R/$O/timeline.csv')))
for x in r[-40:]: print(x['Name'][:60].ljust(60), round(int(x['DurationNs'])/1e3,1), round(int(x['GapBeforeNs'])/1e3,1))
PY
