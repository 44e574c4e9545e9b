#!/bin/bash
# Bench lines of the three training modes (BCE, +KL sampled, +KL full) on one GPU, each under its
# own time limit.   usage (inside gpurun): bash tools/gpu_bench_modes.sh TAG [extra bench args]
TAG=${1:-m}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$TAG; mkdir -p $O
run() {
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
}
run base
run reg --reg 0.1
run full --reg 0.1 --reg-mode full --steps 20 --warmup 3
