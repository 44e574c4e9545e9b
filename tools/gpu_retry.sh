#!/bin/bash
# Run one gpurun command; re-submit ONLY when the infrastructure reports a transient failure
# before anything ran (exit 3 / status=transient).  Never retries a command that ran.
# usage: tools/gpu_retry.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if [ $rc -eq 3 ] || echo "$out" | grep -q "status=transient"; then
    echo "[retry] transient infrastructure failure, waiting 60s"; sleep 60; continue
  fi
  exit $rc
done
exit 3
