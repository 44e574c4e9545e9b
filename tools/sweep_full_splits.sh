cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sw
for sp in 1 2 3 4; do
  CCREC_DX_SPLITS_REG=$sp timeout -k 10 200 python bench.py --reg 0.1 --reg-mode full --steps 10 --warmup 3 --no-cpu-baseline --no-recommend > gpurun_out/sw/sp$sp.log 2>&1 || exit 1
  tail -1 gpurun_out/sw/sp$sp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($sp, round(d['ms_per_step']*1e3,1), d['final_loss'])"
done
