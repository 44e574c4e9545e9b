set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for bm in 128 512; do
  for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    CCREC_NT_BM=$bm timeout -k 10 120 rocprofv3 --pmc $ctr -d $R/gpurun_out/pmc_${bm}_${tag} -o run --output-format csv -- python3 $R/tools/micro/gemm_one.py compute_only > $R/gpurun_out/pmc_${bm}_${tag}.log 2>&1
  done
done
