#!/bin/bash
# PMC passes over the fused output-layer micro (one counter group per run).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/dpmc
mkdir -p $O
for m in 0 7; do
  i=0
  for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    CCREC_DECOUT_DBG=$m N=10 timeout -s KILL 90 rocprofv3 --pmc $ctr -d $O/m${m}_$i -o run --output-format csv -- python3 $R/tools/micro/decout_micro.py > $O/m${m}_$i.log 2>&1 || exit 1
  done
done
echo ok
