#!/bin/bash
# Config-5 kernel change check: the MX-FP8 kernel tests, the fp8 training tests, then the config-5
# line twice (per-kernel event times).  usage: bash tools/gpu_c5k.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-c5k}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -k "fp8 or d1024" --timeout 200 --timeout-method thread > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --d 1024 --dtype fp8 --reg 0.1 --steps 60 --warmup 5 --no-cpu-baseline --no-recommend > $O/c5_$i.log 2>&1 || { tail -20 $O/c5_$i.log; exit 1; }
  tail -1 $O/c5_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
done
