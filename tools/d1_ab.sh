#!/bin/bash
# D1 A/B vs a tagged build: bit-identity of every cc_dec_bce_dw path, then the kernel alone (interleaved)
#   bash tools/d1_ab.sh OUTDIR TAG     (TAG: libccrec_hip_TAG.so, built from the tree to compare against)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$1; T=$2; mkdir -p $O; W=/tmp/d1ab; mkdir -p $W
OLD=$R/cubecobrarecommender_amd/libccrec_hip_$T.so
CCREC_LIB=$OLD timeout -k 10 180 python -u tools/micro/d1_ab.py dump $W/old.npz > $O/dump_old.log 2>&1 || exit 1
timeout -k 10 180 python -u tools/micro/d1_ab.py dump $W/new.npz > $O/dump_new.log 2>&1 || exit 1
python tools/micro/d1_ab.py cmp $W/old.npz $W/new.npz > $O/cmp.log 2>&1; echo "cmp rc $?" >> $O/cmp.log; tail -3 $O/cmp.log
for i in 1 2; do
  CCREC_LIB=$OLD timeout -k 10 120 python -u tools/micro/d1_ab.py time >> $O/time.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/micro/d1_ab.py time >> $O/time.log 2>&1 || exit 1
done
grep dec_bce $O/time.log
