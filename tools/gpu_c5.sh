#!/bin/bash
# Config 5 checks: the fp8 train tests and the d=1024 MX-FP8 +KL bench line; then the default line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-c5}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -k "fp8 or d1024" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u bench.py --d 1024 --dtype fp8 --reg 0.1 --steps 30 --warmup 5 --no-cpu-baseline --no-recommend > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
tail -1 $O/c5.log | cut -c1-600
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/base.log 2>&1 || { tail -20 $O/base.log; exit 1; }
tail -1 $O/base.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1e3,1), d['recommend'])"
