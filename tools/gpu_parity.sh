#!/bin/bash
# Parity tests at the shipped sizes with the observed errors logged (CCREC_PARITY_LOG) so the
# tolerances can be set from measurements.  usage (inside gpurun): bash tools/gpu_parity.sh TAG [pytest args]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=${1:-par}; shift; O=gpurun_out/$T; mkdir -p $O
export CCREC_PARITY_LOG=$R/$O/parity.jsonl
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $O/parity.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $O/parity.log | tail -30
exit $rc
