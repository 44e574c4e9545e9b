#!/bin/bash
# round-3 check 2: KL A/B probes, then the touched GPU tests, then the +KL / config-5 bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t4; mkdir -p $O
bash tools/gpu_klab.sh > $O/klab.log 2>&1 || { tail -5 $O/klab.log; exit 1; }
grep -E "==|rep 2|rep 4" $O/klab.log
timeout -k 10 800 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_mx8.py -q --timeout 200 --timeout-method thread -k "gather or dec_bce or train_steps or full_mode or fused_w1 or adam_pack or clip or dx_splitk or fp8 or quant" > $O/sel.log 2>&1
tail -3 $O/sel.log; grep -E "^FAILED|Error" $O/sel.log | head -5
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"; }
run reg --reg 0.1
run full --reg 0.1 --reg-mode full --steps 20 --warmup 3
run c5 --reg 0.1 --d 1024 --dtype fp8 --steps 50 --warmup 5
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -q --timeout 300 --timeout-method thread > $O/dp.log 2>&1
tail -3 $O/dp.log; grep -E "^FAILED|Error" $O/dp.log | head -5
