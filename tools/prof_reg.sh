#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 "$R/bench.py" --reg 0.1 --steps 50 --warmup 5 --no-cpu-baseline --no-recommend > "$O/prof.log" 2>&1
echo rc $?
find $O/prof -name "*kernel_stats.csv" | head -2
