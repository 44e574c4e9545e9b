bash tools/gpu_run.sh r05zq tests py:tools/run_smoke.py "fullbench:--steps 20 --warmup 5"
