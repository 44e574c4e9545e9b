#!/bin/bash
# d = 512 / 1024 XCD column-sliced E1 gather: kernel tests, the fp8 training tests, then the config-5
# line A/B over CCREC_GATHER_XCDW variants (0 = the previous gather_kernel).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-gw}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gather" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -k "fp8 or d1024 or 512" --timeout 200 --timeout-method thread > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
bash tools/ab_env.sh gw CCREC_GATHER_XCDW=0 CCREC_GATHER_XCDW=44 CCREC_GATHER_XCDW=28 CCREC_GATHER_XCDW=48 -- --d 1024 --dtype fp8 --reg 0.1 --steps 40 --warmup 5
