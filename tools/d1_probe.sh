cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r06w1 /tmp/pb
for v in "" "-DPROBE_OFF"; do n=dec_probe2$( [ -n "$v" ] && echo _off ); hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-honor-nans -I include -I cubecobrarecommender_amd/csrc $v tools/micro/dec_probe2.hip cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o /tmp/pb/$n || exit 1; done
timeout -k 10 60 /tmp/pb/dec_probe2_off > gpurun_out/r06w1/off.log 2>&1 && timeout -k 10 60 /tmp/pb/dec_probe2 > gpurun_out/r06w1/probe.log 2>&1
cat gpurun_out/r06w1/off.log; tail -12 gpurun_out/r06w1/probe.log
