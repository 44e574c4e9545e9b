for v in 22000 2504 5000; do timeout -k 5 120 tools/micro/gpubin/kl_ab $v 16 && timeout -k 5 120 tools/micro/gpubin/kl_ab_s0 $v 16 || exit 1; done
bash tools/gpu_run.sh r05za "tests:tests/test_gpu_train.py -k full_mode" && bash tools/ab_lib.sh old --reg 0.1 --reg-mode full --steps 10 --warmup 3
