bash tools/gpu_run.sh r05zi "tests:tests/test_gpu_dp.py tests/test_gpu_api.py"
