#!/bin/bash
# One GPU-box session: gpu tests, the default bench line, rocprofv3 kernel stats of the same bench,
# and the two PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) for the roofline kernel.
# usage (inside gpurun): bash tools/gpu_round.sh TAG [skip-tests]
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
  tail -3 "$O/gpu_tests.log"
fi
timeout -k 10 300 python -u bench.py > "$O/bench.log" 2>&1
tail -1 "$O/bench.log"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-recommend > "$O/prof_bench.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- \
  python3 "$R/bench.py" --steps 16 --warmup 4 --no-cpu-baseline --no-recommend > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run -- \
  python3 "$R/bench.py" --steps 16 --warmup 4 --no-cpu-baseline --no-recommend > "$O/pmc_write.log" 2>&1
echo done
