#!/bin/bash
# Round-3 closing evidence on one GPU box: the GPU suite, smoke, kernel stats of the four bench lines
# (BCE, +KL sampled, full mode, config 5), the dispatch timeline of the BCE step, PMC passes over the
# BCE line (HBM bytes of the roofline kernel; MFMA), then the bench lines with the traffic attached.
# usage (inside gpurun): bash tools/gpu_r03x.sh [tests|prof|bench|all]
WHAT=${1:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/${TAG:-r03x}; mkdir -p $O
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -3 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "$WHAT" = pmc ]; then
  export TMPDIR=/tmp
  B="$R/bench.py"
  pmc() { n=$1; c=$2; shift 2
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/pmc_$n" -o run -- python3 "$B" --no-cpu-baseline --no-recommend "$@" > "$O/pmc_$n.log" 2>&1) || { echo "pmc $n failed"; tail -5 "$O/pmc_$n.log"; exit 1; }
    python3 "$R/tools/prof_collect.py" pmc "$O/pmc_$n" "$O/pmc_$n.json" || exit 1; echo "pmc $n ok"; }
  pmc fetch FETCH_SIZE --steps 16 --warmup 4
  pmc write WRITE_SIZE --steps 16 --warmup 4
  python3 "$R/tools/traffic_from_pmc.py" "$O/pmc_fetch.json" "$O/pmc_write.json" "$O/traffic_r03x.json" \
    adam_noise_kernel:adam_noise_kernel embed_grad_cs_kernel:embed_grad_cs_kernel || exit 1
  timeout -k 10 400 python -u bench.py --traffic-json $O/traffic_r03x.json > $O/bench_base.log 2>&1 || { tail -5 $O/bench_base.log; exit 1; }
  tail -1 $O/bench_base.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1e3,1), 'us/step', json.dumps(d['roofline']))"
fi
if [ "$WHAT" = prof ] || [ "$WHAT" = all ]; then
  export TMPDIR=/tmp
  B="$R/bench.py"
  stats() { n=$1; shift
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run -- python3 "$B" --no-cpu-baseline --no-recommend "$@" > "$O/prof_$n.log" 2>&1) || { echo "stats $n failed"; tail -5 "$O/prof_$n.log"; exit 1; }
    python3 "$R/tools/prof_collect.py" stats "$O/prof_$n" "$O/stats_$n.csv" || exit 1; echo "stats $n ok"; }
  pmc() { n=$1; c=$2; shift 2
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/pmc_$n" -o run -- python3 "$B" --no-cpu-baseline --no-recommend "$@" > "$O/pmc_$n.log" 2>&1) || { echo "pmc $n failed"; tail -5 "$O/pmc_$n.log"; exit 1; }
    python3 "$R/tools/prof_collect.py" pmc "$O/pmc_$n" "$O/pmc_$n.json" || exit 1; echo "pmc $n ok"; }
  stats base --steps 100 --warmup 10
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/prof_tl" -o run -- python3 "$B" --steps 30 --warmup 5 --no-cpu-baseline --no-recommend > "$O/prof_tl.log" 2>&1) && python3 "$R/tools/prof_collect.py" timeline "$O/prof_tl" "$O/timeline_base.csv" || exit 1
  stats reg --reg 0.1 --steps 100 --warmup 10
  stats full --reg 0.1 --reg-mode full --steps 20 --warmup 3
  stats c5 --dtype fp8 --d 1024 --reg 0.1 --steps 40 --warmup 5
  pmc fetch FETCH_SIZE --steps 16 --warmup 4
  pmc write WRITE_SIZE --steps 16 --warmup 4
  pmc mfma "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" --steps 16 --warmup 4
  python3 "$R/tools/traffic_from_pmc.py" "$O/pmc_fetch.json" "$O/pmc_write.json" "$O/traffic_r03x.json" \
    adam_noise_kernel:adam_noise_kernel embed_grad_cs_kernel:embed_grad_cs_kernel || exit 1
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  TJ=$O/traffic_r03x.json; [ -f $TJ ] || TJ=$R/profiles/traffic_r03x.json
  run() { n=$1; shift; timeout -k 10 400 python -u bench.py --traffic-json $TJ "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 1; }
    tail -1 $O/bench_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', d['value'])"; }
  run base
  run reg --reg 0.1 --no-cpu-baseline --no-recommend
  run full --reg 0.1 --reg-mode full --steps 30 --warmup 3 --no-cpu-baseline --no-recommend
  run c5 --dtype fp8 --d 1024 --reg 0.1 --steps 60 --warmup 5 --no-cpu-baseline --no-recommend
fi
echo done
