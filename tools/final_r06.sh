# Round-6 closing evidence in two gpurun calls (each under gpurun's 20-minute cap):
#   TAG=r06f PART=a bash tools/final_r06.sh   GPU suite, smoke, the headline line (+ CPU baseline), two driver-style lines
#   TAG=r06f PART=b bash tools/final_r06.sh   the other bench lines, the DP lines, rocprof kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
if [ "${PART:-a}" == "a" ]; then
bash tools/gpu_run.sh ${TAG:-r06f}a tests py:tools/run_smoke.py fullbench "fullbench:--steps 20 --warmup 5" "fullbench:--steps 20 --warmup 5"
else
bash tools/gpu_run.sh ${TAG:-r06f}b "bench:--reg 0.1" "bench:--d 1024 --dtype fp8 --reg 0.1" "bench:--reg 0.1 --reg-mode full" "bench:--dtype fp32 --steps 20 --warmup 5" "bench:--force-dp --steps 50 --warmup 10" "bench:--force-dp --dp-graph 0 --steps 50 --warmup 10" "bench:--force-dp --reg 0.1 --steps 50 --warmup 10" "bench:--force-dp --d 1024 --dtype fp8 --reg 0.1 --steps 50 --warmup 10" "prof:--steps 50" "prof:--reg 0.1 --steps 50" "prof:--reg 0.1 --reg-mode full --steps 10 --warmup 3" "prof:--d 1024 --dtype fp8 --reg 0.1 --steps 20 --warmup 5"
fi
