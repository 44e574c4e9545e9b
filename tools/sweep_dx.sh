#!/bin/bash
# dX split-K sweep on the default bench line (same box, interleaved).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/sweep_dx; mkdir -p $O
for rep in 1 2; do
for sp in 16 24 32 44; do
  CCREC_DX_SPLITS=$sp timeout -k 10 200 python bench.py --no-cpu-baseline --no-recommend > $O/sp$sp.log 2>&1 || exit 1
  tail -1 $O/sp$sp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($sp, round(d['ms_per_step']*1e3,1), round(d['kernel_us']['dec_dX'],1))"
done; done
