#!/bin/bash
# One GPU-box session: GPU tests (optional subset), the default bench line, a 2-rank bench
# rehearsal on the one GPU (gloo), each step under its own time limit, stopping at the first failure.
# usage (inside gpurun): bash tools/gpu_session.sh TAG [pytest-args...]
TAG=${1:-s}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "$@" \
  > "$O/gpu_tests.log" 2>&1
rc=$?
grep -E "passed|failed|Error" "$O/gpu_tests.log" | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-600
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline \
  --no-recommend > "$O/bench_dp2.log" 2>&1 || { tail -20 "$O/bench_dp2.log"; exit 1; }
tail -1 "$O/bench_dp2.log" | cut -c1-400
echo done
