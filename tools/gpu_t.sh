cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "fused_regulariser or full_mode or bench_config or match_oracle" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_micro.sh r02k tools/micro/kl_micro.py | head -8
SKIP_TESTS=1 bash tools/gpu_session.sh r02k
