for x in x1 x0 x1 x0; do timeout -k 5 60 tools/micro/gpubin/dwo_diag_$x || exit 1; done
bash tools/gpu_run.sh r05zs "tests:tests/test_gpu_train.py -k full_mode" "tests:tests/test_gpu_fullsize.py -k full_mode"
