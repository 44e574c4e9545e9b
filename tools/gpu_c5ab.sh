#!/bin/bash
# Config-5 A/B: the mx8 GPU tests, the MX-FP8 micro-bench, then the config-5 line under each
# environment assignment given (e.g. "CCREC_DX_SPLITS=16").  usage: bash tools/gpu_c5ab.sh TAG [ENV ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-c5ab}; shift; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -u tools/micro/mx8_bench.py > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
grep us $O/b.log
i=0
for e in "X=0" "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py --d 1024 --dtype fp8 --reg 0.1 --steps 40 --warmup 5 --no-cpu-baseline --no-recommend > $O/c5_$i.log 2>&1 || { tail -20 $O/c5_$i.log; exit 1; }
  tail -1 $O/c5_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $e', round(d['ms_per_step']*1e3,1), 'us/step')"
done
