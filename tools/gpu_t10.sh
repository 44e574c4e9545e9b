#!/bin/bash
# A/B: Wo slices warmed into L2 by the tower forward's extra blocks (CCREC_WO_WARM), BCE bench x2 each
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py -q --timeout 200 --timeout-method thread -k "step_many or fused_w1 or bench_config or train_steps" > $O/sel.log 2>&1; tail -2 $O/sel.log
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_us'] or {}; print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {a: round(b,1) for a,b in k.items()})"; }
for v in 0 1 0 1; do CCREC_WO_WARM=$v run w$v || exit 1; done
