bash tools/gpu_run.sh r05zk "tests:tests/test_gpu_kernels.py -k dx_splitk" "tests:tests/test_gpu_fullsize.py -k full_mode" "tests:tests/test_gpu_train.py -k full_mode"
