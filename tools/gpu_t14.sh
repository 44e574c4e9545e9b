#!/bin/bash
# A/B: W1 Adam operand prefetch across tiles (default lib) vs libccrec_hip_ne.so (EG_EARLY=0)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t14; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py -q --timeout 200 --timeout-method thread -k "fused_w1 or bench_config or step_many" > $O/sel.log 2>&1; tail -1 $O/sel.log
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_us'] or {}; r=d['roofline']; print('$n', round(d['ms_per_step']*1e3,1), 'us/step', 'w1', round(k.get('cc_embed_scatter_bwd',0),1), 'roof', round(r['achieved']), round(r['frac'],3))"; }
NP=$R/cubecobrarecommender_amd/libccrec_hip_ne.so
for v in e np e np; do if [ $v = np ]; then CCREC_LIB=$NP run $v || exit 1; else run $v || exit 1; fi; done
