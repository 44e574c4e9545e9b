#!/bin/bash
# Wo Adam in the tower backward launch: parity (fused vs unfused bits, bench config vs oracle), BCE bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t7; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py -q --timeout 300 --timeout-method thread -k "fused_w1_adam or bench_config" > $O/sel.log 2>&1; tail -3 $O/sel.log
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()}, 'adam', round(d['roofline']['avg_ms']*1e3,1))"; }
run base
run base2
