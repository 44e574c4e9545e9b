cd $GRAFT_REPO_ROOT
bash tools/micro/ab_probe.sh dec_probe2.hip || exit 1
cp cubecobrarecommender_amd/csrc/decout.hip /tmp/x.hip
bash tools/gpu_bench_modes.sh m2 || exit 1
mkdir -p gpurun_out/t2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t2/t.log 2>&1; rc=$?
tail -3 gpurun_out/t2/t.log; exit $rc
