#!/bin/bash
# tests of the deferred output-layer Adam + bench A/B of its placement: bash tools/fwd_ab.sh OUT
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  -k "fused_w1_adam or step_many_multi" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for reg in 0 0.1; do
  for i in 1 2; do
    for f in 0 1; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend --reg $reg --wo-fwd $f > $O/b_r${reg}_f${f}_$i.log 2>&1 || { tail -20 $O/b_r${reg}_f${f}_$i.log; exit 1; }
      tail -1 $O/b_r${reg}_f${f}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('reg $reg wo_fwd $f', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k, v in d.get('kernel_us', {}).items()})"
    done
  done
done
