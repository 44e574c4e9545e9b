#!/bin/bash
# sweep: fraction of Wo's Adam in the tower backward launch (the rest beside F in the Adam launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t8; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "fused_w1_adam" > $O/sel.log 2>&1; tail -2 $O/sel.log
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_us'] or {}; print('$n', round(d['ms_per_step']*1e3,1), 'us/step', 'tbwd', round(k.get('cc_tower_bwd',0),1), 'adam', round(k.get('cc_adam_dense',0),1), 'w1', round(k.get('cc_embed_scatter_bwd',0),1))"; }
for f in ${FRACS:-0 0.4 0.5 0.6 0.7 0.8 1.0}; do CCREC_WO_TOWER_FRAC=$f run f$f || exit 1; done
