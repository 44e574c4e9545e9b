#!/bin/bash
# Wide (d > 256) tower kernels: tower tests, the config-5 train tests, then the config-5 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-wide}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -x -q --timeout 120 --timeout-method thread > $O/tower.log 2>&1 || { tail -40 $O/tower.log; exit 1; }
tail -2 $O/tower.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_mx8.py -m gpu -x -q -k "fp8 or d1024 or mx8 or 512" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u bench.py --d 1024 --dtype fp8 --reg 0.1 --steps 30 --warmup 5 --no-cpu-baseline --no-recommend > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
