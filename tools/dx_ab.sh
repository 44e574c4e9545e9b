#!/bin/bash
# dX split-K alone at the bench shape across library builds: bash tools/dx_ab.sh OUT TAG...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$1; shift; mkdir -p $O
for i in 1 2; do
  for t in "$@"; do
    L=$R/cubecobrarecommender_amd/libccrec_hip.so; [ $t != prod ] && L=$R/cubecobrarecommender_amd/libccrec_hip_$t.so
    echo "== $t" >> $O/dx.log
    SPLITS="16 32" CCREC_LIB=$L timeout -k 10 120 python -u tools/micro/dx_split_micro.py >> $O/dx.log 2>&1 || exit 1
  done
done
