#!/bin/bash
# MX-FP8 GEMM kernels: the mx8 GPU tests and the fp8 training tests, tools/micro/mx8_bench.py on
# the 256 x 256 kernel and the 128 x 128 kernel (CCREC_MX8_GEMM=128), then the config-5 bench line
# both ways.  usage: bash tools/gpu_mx8.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-mx}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q -k "fp8 or d1024" --timeout 200 --timeout-method thread > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
timeout -k 10 200 python -u tools/micro/mx8_bench.py > $O/b256.log 2>&1 || { tail -20 $O/b256.log; exit 1; }
CCREC_MX8_GEMM=128 timeout -k 10 200 python -u tools/micro/mx8_bench.py > $O/b128.log 2>&1 || { tail -20 $O/b128.log; exit 1; }
paste $O/b256.log $O/b128.log | grep us
for k in 256 128; do
  CCREC_MX8_GEMM=$k timeout -k 10 300 python -u bench.py --d 1024 --dtype fp8 --reg 0.1 --steps 40 --warmup 5 --no-cpu-baseline --no-recommend > $O/c5_$k.log 2>&1 || { tail -20 $O/c5_$k.log; exit 1; }
  tail -1 $O/c5_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $k', round(d['ms_per_step']*1e3,1), 'us/step')"
done
