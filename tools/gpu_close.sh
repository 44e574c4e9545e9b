#!/bin/bash
# Closing evidence at the head: GPU suite, smoke, the default bench line, the config-5 line, and the
# rocprofv3 kernel stats of the default line.  usage (inside gpurun): bash tools/gpu_close.sh TAG
TAG=${1:-close}; R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python -u bench.py > "$O/bench.log" 2>&1 || { tail -5 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
timeout -k 10 300 python -u bench.py --d 1024 --dtype fp8 --reg 0.1 --steps 60 --warmup 5 --no-cpu-baseline --no-recommend > "$O/c5.log" 2>&1 || { tail -5 "$O/c5.log"; exit 1; }
tail -1 "$O/c5.log" | cut -c1-200
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-recommend > "$O/prof_bench.log" 2>&1 || { tail -5 "$O/prof_bench.log"; exit 1; }
python3 "$R/tools/prof_collect.py" stats "$O/prof" "$O/base_kernel_stats.csv"
echo done
