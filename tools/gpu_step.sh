#!/bin/bash
# Round-2 step changes: tower + W1-gradient kernel tests, tower micro, train / full-size / DP tests,
# then the three bench modes.   usage (inside gpurun): bash tools/gpu_step.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=${1:-st}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_kernels.py -x -q -k "tower or packed or embed_grad" --timeout 120 --timeout-method thread > $O/k.log 2>&1 || { tail -40 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 5 60 tools/micro/gpubin/tower_probe > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
tail -2 $O/probe.log
timeout -k 5 120 python tools/micro/tower_micro.py 2>&1 | grep -v amdgpu.ids > $O/micro.log || exit 1
cat $O/micro.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/gpu_bench_modes.sh $T
