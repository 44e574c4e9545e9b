#!/bin/bash
# two-range Adam placement: parity (bit-identity fused/unfused at reg 0 / 0.1; bench configs vs oracle), sweeps
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t15; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_api.py -q --timeout 200 --timeout-method thread -k "fused_w1 or bench_config or step_many or fit" > $O/sel.log 2>&1; tail -1 $O/sel.log
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_us'] or {}; print('$n', round(d['ms_per_step']*1e3,1), 'us/step', 'tbwd', round(k.get('cc_tower_bwd',0),1), 'adam', round(k.get('cc_adam_dense',0),1), 'w1', round(k.get('cc_embed_scatter_bwd',0),1))"; }
run base
for f in ${FRACS:-0 0.3 0.45 0.6}; do CCREC_WO_TOWER_FRAC=$f run reg$f --reg 0.1 || exit 1; done
