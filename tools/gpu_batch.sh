bash tools/gpu_run.sh r05zj tests py:tools/run_smoke.py fullbench "fullbench:--steps 20 --warmup 5" "bench:--force-dp --steps 50 --warmup 10"
