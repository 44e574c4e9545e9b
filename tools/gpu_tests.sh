#!/bin/bash
# GPU test suite only (one process, per-test timeout); log under gpurun_out/<tag>/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tests}
mkdir -p "$O"
cd "$R"
shift
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread "$@" \
  > "$O/gpu_tests.log" 2>&1
rc=$?
grep -E "passed|failed|Error|error" "$O/gpu_tests.log" | tail -30
exit $rc
