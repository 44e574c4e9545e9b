#!/bin/bash
# Quick A/B: the named kernel tests, then the BCE and +KL bench lines.  usage: bash tools/gpu_quick.sh TAG "pytest -k expr"
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=${1:-q}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_kernels.py -x -q -k "${2:-embed_grad}" --timeout 120 --timeout-method thread > $O/k.log 2>&1 || { tail -40 $O/k.log; exit 1; }
tail -1 $O/k.log
run() {
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
}
run base
run reg --reg 0.1
