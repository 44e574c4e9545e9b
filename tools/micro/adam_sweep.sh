set -e
mkdir -p gpurun_out/as
for nb in 2048 4096 100000; do
  for pf in 1 0; do
    echo "blocks=$nb prefetch=$pf" >> gpurun_out/as/b.log
    CCREC_ADAM_BLOCKS=$nb CCREC_PREFETCH_NOISE=$pf timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-recommend --steps 100 2>/dev/null | python -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(b['ms_per_step']*1e3, b['roofline']['avg_ms']*1e3, b['kernel_ms_eager'].get('cc_adam_dense'))" >> gpurun_out/as/b.log
  done
done
