#!/bin/bash
# A/B two builds of the library on the bench (interleaved runs): bash tools/ab_lib.sh TAG [bench args]
# (library variants: CCREC_BUILD_TAG=x CCREC_EXTRA_FLAGS=... python -m cubecobrarecommender_amd.build)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=$1; shift; O=gpurun_out/ab_$T; mkdir -p $O
for i in 1 2; do
  for v in base $T; do
    L=cubecobrarecommender_amd/libccrec_hip.so; [ $v != base ] && L=cubecobrarecommender_amd/libccrec_hip_$v.so
    CCREC_LIB=$R/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/$v$i.log 2>&1 || { tail -20 $O/$v$i.log; exit 1; }
    tail -1 $O/$v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3,1), 'us/step', d['kernel_us'])"
  done
done
