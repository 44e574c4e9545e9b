#!/bin/bash
# A/B runtime variants of one library build on the bench (interleaved, twice):
#   bash tools/ab_env.sh TAG "VAR=a" "VAR=b" ... -- [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=$1; shift; O=gpurun_out/ab_$T; mkdir -p $O
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
for i in 1 2; do
  k=0
  for v in "${V[@]}"; do
    k=$((k+1))
    env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/v$k.$i.log 2>&1 || { tail -20 $O/v$k.$i.log; exit 1; }
    tail -1 $O/v$k.$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
  done
done
