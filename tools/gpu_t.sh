cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread -k "fused_regulariser or full_mode or bench_config or match_oracle or sharded" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_micro.sh r02n tools/micro/kl_micro.py | head -6
