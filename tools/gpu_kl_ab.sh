cd $GRAFT_REPO_ROOT
bash tools/micro/ab_probe.sh kl_probe2.hip || exit 1
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t/t.log 2>&1; rc=$?
tail -5 gpurun_out/t/t.log; exit $rc
