#!/bin/bash
# round-3 check: the d = 512 training cases (verbose), the kernel/training selection, the full-mode bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "train_steps and 512" --tb=short > $O/t512.log 2>&1
grep -E "Error|assert|passed|failed" $O/t512.log | tail -12
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "(gather or dec_bce or full_mode or fused_w1 or adam_pack or clip or dx_splitk) and not (train_steps and 512)" > $O/sel.log 2>&1
tail -3 $O/sel.log
timeout -k 10 300 python -u bench.py --reg 0.1 --reg-mode full --steps 20 --warmup 3 --no-cpu-baseline --no-recommend > $O/full.log 2>&1 || { tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
