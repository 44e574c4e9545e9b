#!/bin/bash
# W1-gradient change check: kernel tests, train / full-size / DP tests, then the bench modes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${1:-eg}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "embed_grad" --timeout 120 --timeout-method thread > $O/k.log 2>&1 || { tail -40 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/gpu_bench_modes.sh ${1:-eg}
