#!/bin/bash
# One GPU-box session: GPU tests (optional pytest args), then the bench lines: default (configs[1]),
# +KL (configs[2]), +KL full mode, and a 2-rank rehearsal on the one GPU (gloo).  Every step under its
# own time limit; the script stops at the first failure.
# usage (inside gpurun): bash tools/gpu_session.sh TAG [pytest-args...]     (SKIP_TESTS=1 to skip)
TAG=${1:-s}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "$@" \
    > "$O/gpu_tests.log" 2>&1
  rc=$?
  grep -E "passed|failed|Error" "$O/gpu_tests.log" | tail -15
  [ $rc -ne 0 ] && exit $rc
fi
run() {  # name, args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > "$O/bench_$n.log" 2>&1 || { tail -20 "$O/bench_$n.log"; exit 1; }
  tail -1 "$O/bench_$n.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['n_gpus'], round(d['value']), 'cubes/s', round(d['ms_per_step']*1e3,1), 'us/step', d['final_loss'])"
}
run base
run reg --reg 0.1 --no-cpu-baseline --no-recommend
run full --reg 0.1 --reg-mode full --steps 30 --warmup 5 --no-cpu-baseline --no-recommend
run dp2 --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline --no-recommend
echo done
