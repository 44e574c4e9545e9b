#!/bin/bash
# Full-mode regulariser evidence: the bench line, rocprofv3 kernel stats, and
# PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA MOPS / busy) each in its own run; then the 2-rank DP
# rehearsal on this one GPU over gloo with per-kernel times.  usage: bash tools/gpu_full_prof.sh TAG
TAG=${1:-fp}; R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py"
cd $R
timeout -k 10 300 python -u bench.py --reg 0.1 --reg-mode full --steps 20 --warmup 3 --no-cpu-baseline --no-recommend > $O/bench_full.log 2>&1 || { tail -5 $O/bench_full.log; exit 1; }
tail -1 $O/bench_full.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full', round(d['ms_per_step']*1e3,1), 'us/step')"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_full -o run -- python3 $B --reg 0.1 --reg-mode full --steps 10 --warmup 3 --no-cpu-baseline --no-recommend > $O/prof_full.log 2>&1 || { echo stats failed; exit 1; }
python3 $R/tools/prof_collect.py stats $O/prof_full $O/stats_full.csv || exit 1
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"; do
  n=$(echo $c | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/pmc_$n -o run -- python3 $B --reg 0.1 --reg-mode full --steps 6 --warmup 2 --no-cpu-baseline --no-recommend > $O/pmc_$n.log 2>&1 || { echo pmc $n failed; exit 1; }
  python3 $R/tools/prof_collect.py pmc $O/pmc_$n $O/pmc_full_$n.json || exit 1
  echo pmc $n ok
done
cd $R
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-cpu-baseline --no-recommend > $O/bench_dp2.log 2>&1 || { tail -5 $O/bench_dp2.log; exit 1; }
tail -1 $O/bench_dp2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dp2', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
echo done
