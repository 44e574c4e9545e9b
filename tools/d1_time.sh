#!/bin/bash
# D1 alone at the bench shape, interleaved across library builds: bash tools/d1_time.sh OUT TAG...
# (TAG "prod" = libccrec_hip.so, else libccrec_hip_TAG.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$1; shift; mkdir -p $O
for i in 1 2; do
  for t in "$@"; do
    L=$R/cubecobrarecommender_amd/libccrec_hip.so; [ $t != prod ] && L=$R/cubecobrarecommender_amd/libccrec_hip_$t.so
    CCREC_LIB=$L timeout -k 10 120 python -u tools/micro/d1_ab.py time >> $O/time.log 2>&1 || exit 1
  done
done
