#!/bin/bash
# rocprofv3 kernel stats of the config-5 line (d=1024, MX-FP8 decoder / regulariser GEMMs, +KL).
# usage (inside gpurun): bash tools/prof_c5.sh TAG [extra bench args]
TAG=${1:-c5p}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c5" -o run -- \
  python3 "$R/bench.py" --d 1024 --dtype fp8 --reg 0.1 --steps 30 --warmup 5 --no-cpu-baseline --no-recommend "$@" \
  > "$O/prof_c5.log" 2>&1 || { echo "stats c5 failed"; tail -5 "$O/prof_c5.log"; exit 1; }
python3 "$R/tools/prof_collect.py" stats "$O/prof_c5" "$O/stats_c5.csv" || exit 1
tail -1 "$O/prof_c5.log" | cut -c1-400
