#!/bin/bash
# A/B of several library builds on the bench (interleaved, two rounds):
#   bash tools/ab_libs.sh OUT "TAG1 TAG2 ..." [bench args]   (TAG prod = libccrec_hip.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/$1; T=$2; shift 2; mkdir -p $O
for i in 1 2; do
  for v in $T; do
    L=$R/cubecobrarecommender_amd/libccrec_hip.so; [ $v != prod ] && L=$R/cubecobrarecommender_amd/libccrec_hip_$v.so
    CCREC_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/$v$i.log 2>&1 || { tail -20 $O/$v$i.log; exit 1; }
    tail -1 $O/$v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v, 1) for k, v in d['kernel_us'].items()})"
  done
done
