#!/bin/bash
# Profiling session on one GPU box: rocprofv3 kernel stats of the bench lines (BCE, +KL sampled,
# +KL full mode), then PMC passes over the BCE line, one run per pass (MI355X_MICROARCH.md §HBM:
# FETCH_SIZE and WRITE_SIZE in separate passes; MFMA MOPS / busy cycles in a third).
# usage (inside gpurun): bash tools/gpu_prof.sh TAG [stats|pmc|all] [extra bench args...]
TAG=${1:-p}; WHAT=${2:-all}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py"
stats() {  # name, bench args...
  n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run -- \
    python3 "$B" --no-cpu-baseline --no-recommend "$@" > "$O/prof_$n.log" 2>&1 || { echo "stats $n failed"; tail -5 "$O/prof_$n.log"; exit 1; }
  python3 "$R/tools/prof_collect.py" stats "$O/prof_$n" "$O/stats_$n.csv" || exit 1
  tail -1 "$O/prof_$n.log" | cut -c1-200
  echo "stats $n ok"
}
pmc() {  # name, counters, bench args...
  n=$1; c=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$O/pmc_$n" -o run -- \
    python3 "$B" --no-cpu-baseline --no-recommend "$@" > "$O/pmc_$n.log" 2>&1 || { echo "pmc $n failed"; tail -5 "$O/pmc_$n.log"; exit 1; }
  python3 "$R/tools/prof_collect.py" pmc "$O/pmc_$n" "$O/pmc_$n.json" || exit 1
  echo "pmc $n ok"
}
if [ "$WHAT" = stats ] || [ "$WHAT" = all ]; then
  stats base --steps 100 --warmup 10 "$@"
  stats reg --reg 0.1 --steps 100 --warmup 10 "$@"
  stats full --reg 0.1 --reg-mode full --steps 20 --warmup 3 "$@"
fi
if [ "$WHAT" = pmc ] || [ "$WHAT" = all ]; then
  pmc fetch FETCH_SIZE --steps 16 --warmup 4 "$@"
  pmc write WRITE_SIZE --steps 16 --warmup 4 "$@"
  pmc mfma "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" --steps 16 --warmup 4 "$@"
  pmc regfetch FETCH_SIZE --reg 0.1 --steps 16 --warmup 4 "$@"
  pmc regmfma "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" --reg 0.1 --steps 16 --warmup 4 "$@"
fi
echo done
