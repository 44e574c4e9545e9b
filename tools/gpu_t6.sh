#!/bin/bash
# full-mode bench: A/B of the dX kernel's dZ cache policy is in the library; KL probes; bench full
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "dx_splitk or full_mode or clip or train_steps" > $O/sel.log 2>&1; tail -2 $O/sel.log
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"; }
run full --reg 0.1 --reg-mode full --steps 20 --warmup 3
run reg --reg 0.1
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_full -o run -- python3 $R/bench.py --reg 0.1 --reg-mode full --steps 10 --warmup 3 --no-cpu-baseline --no-recommend > $R/$O/prof_full.log 2>&1 || exit 1
python3 $R/tools/prof_collect.py stats $R/$O/prof_full $R/$O/stats_full.csv && head -4 $R/$O/stats_full.csv | cut -c1-150
