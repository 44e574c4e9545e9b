#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over the D1 / D2 probe binaries: where the waves of
# dec_bce_dw_kernel, kl_stats_kernel and kl_main_kernel spend their cycles.
# usage (inside gpurun): bash tools/pmc_probe.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/$1; mkdir -p $O tools/micro/bin
F="-O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc"
for p in dec_probe2 kl_probe2; do
  hipcc $F tools/micro/$p.hip cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/$p 2>/dev/null || exit 1
done
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_EXP SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VALU_MFMA_MOPS_BF16"; do
  i=$((i+1))
  for p in dec_probe2 kl_probe2; do
    timeout -s KILL 60 rocprofv3 --pmc $c -d $O/pmc_${p}_$i -o run -- $R/tools/micro/bin/$p > $O/pmc_${p}_$i.log 2>&1 && \
      python3 tools/prof_collect.py pmc $O/pmc_${p}_$i $O/pmc_${p}_$i.json || echo "pass $i $p failed"
  done
done
echo done
