bash tools/gpu_run.sh r05h2 "py:tools/run_smoke.py" "fullbench:--steps 20 --warmup 5" "prof:" 
