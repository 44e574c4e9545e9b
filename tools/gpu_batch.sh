for s in 4 2 8; do timeout -k 5 60 tools/micro/gpubin/dx_diag_0 $s || exit 1; done
timeout -k 5 60 tools/micro/gpubin/dx_diag_old 4 || exit 1
bash tools/gpu_run.sh r05z7 "tests:tests/test_gpu_kernels.py -k dx_splitk" "tests:tests/test_gpu_train.py -k full_mode" && bash tools/ab_lib.sh old --reg 0.1 --reg-mode full --steps 10 --warmup 3
