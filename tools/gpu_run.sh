#!/bin/bash
# One gpurun session, parameterised (replaces the per-experiment scripts of rounds 1-3):
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
# STEP is one of
#   tests[:<pytest args>]     GPU tests (default: the whole -m gpu suite; args replace 'tests')      -> $O/tests_<i>.log
#   bench[:<bench.py args>]   one bench line                                   -> $O/bench_<i>.log
#   prof[:<bench.py args>]    rocprofv3 --kernel-trace --stats of a bench run  -> $O/prof_<i>/
#   pmc:<C1,C2,..>[:<args>]   one rocprofv3 --pmc pass of a short bench run    -> $O/pmc_<i>.json (per-kernel averages)
#   pmcx:<C1,C2,..>:<prog>    one rocprofv3 --pmc pass over a built probe binary -> $O/pmc_<i>.json
#   py:<script args>          python -u <script args>                          -> $O/py_<i>.log
#   cmd:<command>             any command (a built probe binary)               -> $O/cmd_<i>.log
# Every GPU step runs under its own time limit; the first failing step ends the session.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p "$O"
export CCREC_PARITY_LOG=$O/parity.jsonl
i=0
summ() { python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().strip().splitlines() if l.startswith('{')][-1])
k = d.get('kernel_us') or {}
r = d.get('roofline') or {}
print(round(d['ms_per_step'] * 1e3, 1), 'us/step', d['config']['workload'][:60], '| roof', r.get('tick'),
      round(r.get('frac') or 0, 3), '|', {a: round(b, 1) for a, b in k.items()})
if 'dp' in d:
    print('dp', json.dumps(d['dp']))
PY
}
for st in "$@"; do
  i=$((i + 1)); kind=${st%%:*}; arg=${st#*:}; [ "$arg" == "$st" ] && arg=""
  case $kind in
    tests)
      eval "timeout -k 10 1000 python -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 300 --timeout-method thread" \
        > "$O/tests_$i.log" 2>&1; rc=$?; tail -3 "$O/tests_$i.log"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|error" "$O/tests_$i.log" | tail -20; exit $rc; } ;;
    bench)
      timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-recommend $arg > "$O/bench_$i.log" 2>&1 \
        || { tail -30 "$O/bench_$i.log"; exit 1; }
      summ "$O/bench_$i.log" ;;
    fullbench)
      timeout -k 10 400 python -u bench.py $arg > "$O/bench_$i.log" 2>&1 || { tail -30 "$O/bench_$i.log"; exit 1; }
      summ "$O/bench_$i.log" ;;
    prof)
      ( export TMPDIR=/tmp; cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$i" -o run -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-recommend $arg > "$O/prof_$i.log" 2>&1 ) \
        || { tail -30 "$O/prof_$i.log"; exit 1; }
      summ "$O/prof_$i.log" ;;
    pmc)
      c=${arg%%:*}; a=${arg#*:}; [ "$a" == "$arg" ] && a=""
      ( export TMPDIR=/tmp; cd /tmp && timeout -s KILL 150 rocprofv3 --pmc ${c//,/ } -d "$O/pmc_$i" -o run -- \
        python3 "$R/bench.py" --steps 16 --warmup 4 --no-cpu-baseline --no-recommend $a > "$O/pmc_$i.log" 2>&1 ) \
        || { tail -30 "$O/pmc_$i.log"; exit 1; }
      python tools/prof_collect.py pmc "$O/pmc_$i" "$O/pmc_$i.json" && echo "pmc $c ok" ;;
    pmcx)
      c=${arg%%:*}; a=${arg#*:}
      ( export TMPDIR=/tmp; cd /tmp && timeout -s KILL 90 rocprofv3 --pmc ${c//,/ } -d "$O/pmc_$i" -o run -- \
        "$R/$a" > "$O/pmc_$i.log" 2>&1 ) || { tail -30 "$O/pmc_$i.log"; exit 1; }
      python tools/prof_collect.py pmc "$O/pmc_$i" "$O/pmc_$i.json" && echo "pmc $c ok" ;;
    py)
      timeout -k 10 600 python -u $arg > "$O/py_$i.log" 2>&1 || { tail -30 "$O/py_$i.log"; exit 1; }
      tail -15 "$O/py_$i.log" ;;
    cmd)
      timeout -k 10 300 $arg > "$O/cmd_$i.log" 2>&1 || { tail -30 "$O/cmd_$i.log"; exit 1; }
      tail -12 "$O/cmd_$i.log" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "session $TAG done"
