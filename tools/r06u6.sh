#!/bin/bash
# D1 mask image: bit-identity of every path, kernel timing, tests, bench A/B of the Adam placement
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$1; mkdir -p $O; T=/tmp/d1ab; mkdir -p $T
timeout -k 10 180 python -u tools/micro/d1_ab.py dump $T/new.npz > $O/dump.log 2>&1 || exit 1
python tools/micro/d1_ab.py cmp $T/new.npz > $O/cmp.log 2>&1; echo "cmp rc $?" >> $O/cmp.log; tail -2 $O/cmp.log
for i in 1 2; do timeout -k 10 120 python -u tools/micro/d1_ab.py time >> $O/time.log 2>&1 || exit 1; done
grep dec_bce $O/time.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_fullsize.py \
  -k "dec_bce or mask_image or fused_w1 or step_many or bench_configuration" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for reg in 0 0.1; do
  for i in 1 2; do
    for f in 0 1; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend --reg $reg --wo-fwd $f > $O/b_r${reg}_f${f}_$i.log 2>&1 || { tail -20 $O/b_r${reg}_f${f}_$i.log; exit 1; }
      tail -1 $O/b_r${reg}_f${f}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('reg $reg wo_fwd $f', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k, v in d.get('kernel_us', {}).items()})"
    done
  done
done
