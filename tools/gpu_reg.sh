#!/bin/bash
# gpu tests + the +KL bench (configs[2]) and its rocprofv3 kernel stats.
set -e
TAG=${1:-reg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
timeout -k 10 300 python -u bench.py --reg 0.1 --no-cpu-baseline --no-recommend > "$O/bench_reg.log" 2>&1
tail -1 "$O/bench_reg.log" | cut -c1-400
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_reg" -o run -- \
  python3 "$R/bench.py" --reg 0.1 --no-cpu-baseline --no-recommend > "$O/prof_reg.log" 2>&1
echo done
