cd $GRAFT_REPO_ROOT
for sp in 16 24 32 48; do
  CCREC_DX_SPLITS=$sp timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-recommend > gpurun_out/sp$sp.log 2>&1 || exit 1
  tail -1 gpurun_out/sp$sp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($sp, round(d['ms_per_step']*1e3,1), d['kernel_us']['dec_dX'])"
done
