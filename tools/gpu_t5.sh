#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t5; mkdir -p $O
bash tools/gpu_klab.sh > $O/klab.log 2>&1 || { tail -5 $O/klab.log; exit 1; }
grep -E "==|rep 2|rep 4" $O/klab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -q --timeout 300 --timeout-method thread > $O/dp.log 2>&1
tail -3 $O/dp.log; grep -E "^FAILED|Error" $O/dp.log | head -5
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"; }
run base
run reg --reg 0.1
run full --reg 0.1 --reg-mode full --steps 20 --warmup 3
run dp2 --gpus 2 --backend gloo --steps 10 --warmup 3
