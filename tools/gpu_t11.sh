#!/bin/bash
# A/B: waves per packed tower-dW job (CCREC_DW_WAVES 1 / 2 / 4 / 8), BCE bench; dW tests
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/t11; mkdir -p $O
for v in 1 4 8; do CCREC_DW_WAVES=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_tower.py -q --timeout 100 --timeout-method thread -k "packed_dw" > $O/t_$v.log 2>&1; echo "dw_waves=$v: $(tail -1 $O/t_$v.log)"; done
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_us'] or {}; print('$n', round(d['ms_per_step']*1e3,1), 'us/step', {a: round(b,1) for a,b in k.items()})"; }
for v in 1 4 8 2 1 4; do CCREC_DW_WAVES=$v run w$v || exit 1; done
export TMPDIR=/tmp
for v in 1 4 8; do (cd /tmp && CCREC_DW_WAVES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$v -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-recommend > $R/$O/prof_$v.log 2>&1) && python3 $R/tools/prof_collect.py stats $R/$O/prof_$v $R/$O/stats_$v.csv && grep -i "tower_dw" $R/$O/stats_$v.csv | cut -d, -f1,2,4 | cut -c1-160; done
