R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p tools/micro/bin gpurun_out/klp
F="-O3 -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc"
for p in kl_probe_full kl_probe2; do hipcc $F tools/micro/$p.hip cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/$p || exit 1; done
timeout -k 5 120 tools/micro/bin/kl_probe_full > gpurun_out/klp/full.txt 2>&1 && timeout -k 5 60 tools/micro/bin/kl_probe2 > gpurun_out/klp/s.txt 2>&1
cat gpurun_out/klp/full.txt gpurun_out/klp/s.txt
