#!/bin/bash
# bench A/B of the deferred output-layer Adam fraction: bash tools/fwd_frac.sh OUT REG FRAC...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$1; reg=$2; shift 2; mkdir -p $O
for i in 1 2; do
  for f in 0 "$@"; do
    w=1; [ "$f" = 0 ] && w=0
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend --reg $reg --wo-fwd $w --wo-fwd-frac $f > $O/b_r${reg}_$f_$i.log 2>&1 || { tail -20 $O/b_r${reg}_$f_$i.log; exit 1; }
    tail -1 $O/b_r${reg}_$f_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('reg $reg frac $f', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k, v in d.get('kernel_us', {}).items()})"
  done
done
