R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/gpu_run.sh r04aj tests py:tools/run_smoke.py fullbench "fullbench:--steps 20 --warmup 5" "fullbench:--steps 20 --warmup 5" "bench:--reg 0.1" "bench:--d 1024 --dtype fp8 --reg 0.1" "bench:--reg 0.1 --reg-mode full" "prof:--steps 50"
