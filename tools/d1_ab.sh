#!/bin/bash
# D1 A/B on the GPU box: bit-identity of every cc_dec_bce_dw path vs libccrec_hip_old.so, then the
# kernel alone at the bench shape (interleaved), then the D1 tests.  bash tools/d1_ab.sh OUTDIR
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$1; mkdir -p $O; T=/tmp/d1ab; mkdir -p $T
OLD=$R/cubecobrarecommender_amd/libccrec_hip_old.so
CCREC_LIB=$OLD timeout -k 10 180 python -u tools/micro/d1_ab.py dump $T/old.npz > $O/dump_old.log 2>&1 || exit 1
timeout -k 10 180 python -u tools/micro/d1_ab.py dump $T/new.npz > $O/dump_new.log 2>&1 || exit 1
python tools/micro/d1_ab.py cmp $T/old.npz $T/new.npz > $O/cmp.log 2>&1; echo "cmp rc $?" >> $O/cmp.log
for i in 1 2; do
  CCREC_LIB=$OLD timeout -k 10 120 python -u tools/micro/d1_ab.py time >> $O/time.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/micro/d1_ab.py time >> $O/time.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dec_bce" > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
