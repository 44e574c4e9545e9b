#!/bin/bash
# Config 5's output-layer Adam in the MX-FP8 dW epilogue: bit-identity vs the unfused placement,
# the fp8 / MX tests, the full-size config-5 oracle test, then the config-5 line twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-wo8}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v -k "fp8_fused_output_adam" --timeout 200 --timeout-method thread > $O/t0.log 2>&1 || { tail -40 $O/t0.log; exit 1; }
tail -1 $O/t0.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py tests/test_gpu_train.py -m gpu -x -q -k "mx8 or fp8 or d1024" --timeout 200 --timeout-method thread > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k "config5" --timeout 300 --timeout-method thread > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --d 1024 --dtype fp8 --reg 0.1 --steps 60 --warmup 5 --no-cpu-baseline --no-recommend > $O/c5_$i.log 2>&1 || { tail -20 $O/c5_$i.log; exit 1; }
  tail -1 $O/c5_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
done
