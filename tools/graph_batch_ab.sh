#!/bin/bash
# HIP graph launch batching A/B on the bench (dev tool): the step-boundary gaps seen in the
# kernel trace (every 18th kernel node of the multi-step graph) against the HIP runtime's graph
# packet batch settings.  bash tools/graph_batch_ab.sh TAG [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=$1; shift; O=gpurun_out/gb_$T; mkdir -p $O
for i in 1 2; do
  for v in "" "DEBUG_HIP_GRAPH_BATCH_SIZE=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "DEBUG_HIP_GRAPH_BATCH_SIZE=1024" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
    tag=${v:-default}; tag=${tag//=/_}
    env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/$tag$i.log 2>&1 || { tail -20 $O/$tag$i.log; exit 1; }
    tail -1 $O/$tag$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('${tag}', round(d['ms_per_step']*1e3,1), 'us/step')"
  done
done
