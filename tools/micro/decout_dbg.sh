cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dbg && rm -f gpurun_out/dbg/t.log
for v in ${VS:-22000}; do for m in ${MODES:-0 7 15 8}; do V=$v CCREC_DECOUT_DBG=$m timeout -k 10 60 python tools/micro/decout_micro.py >> gpurun_out/dbg/t.log 2>&1 || exit 1; done; done
grep dec_bce gpurun_out/dbg/t.log
