cd $GRAFT_REPO_ROOT
bash tools/micro/ab_probe.sh dec_probe2.hip 2 || exit 1
mkdir -p gpurun_out/t4
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dec_bce or bench_configuration or train_steps" > gpurun_out/t4/t.log 2>&1; rc=$?
tail -3 gpurun_out/t4/t.log; exit $rc
