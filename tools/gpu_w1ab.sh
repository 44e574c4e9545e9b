#!/bin/bash
# A/B of library builds (abvar/libvar_<tag>.so, made with CCREC_EXTRA_FLAGS) on the config-5 line,
# interleaved twice.  usage: bash tools/gpu_w1ab.sh TAG v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=$1; shift; O=gpurun_out/ab_$T; mkdir -p $O
for i in 1 2; do
  for v in base "$@"; do
    L=$R/cubecobrarecommender_amd/libccrec_hip.so; [ $v != base ] && L=$R/abvar/libvar_$v.so
    CCREC_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend --d 1024 --dtype fp8 --reg 0.1 --steps 60 --warmup 5 > $O/$v$i.log 2>&1 || { tail -20 $O/$v$i.log; exit 1; }
    tail -1 $O/$v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items() if k in ('cc_embed_scatter_bwd','cc_adam_dense')})"
  done
done
