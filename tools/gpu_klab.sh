#!/bin/bash
# A/B of decreg.hip (working tree vs tools/micro/ab_orig/decreg.hip) on the KL phase probes: full mode
# (kl_probe_full) and the sampled +KL shape (kl_probe2)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p tools/micro/bin gpurun_out/klab
F="-O3 -std=c++17 --offload-arch=gfx950 -I include"
for p in kl_probe_full kl_probe2; do
  hipcc $F -I cubecobrarecommender_amd/csrc tools/micro/$p.hip cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/${p}_new 2>/dev/null || exit 1
  hipcc $F -I tools/micro/ab_orig -I cubecobrarecommender_amd/csrc tools/micro/$p.hip cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/${p}_orig 2>/dev/null || exit 1
done
for v in orig new orig new; do
  echo "== $v"
  timeout -k 5 120 tools/micro/bin/kl_probe_full_$v | tail -1 || exit 1
  timeout -k 5 60 tools/micro/bin/kl_probe2_$v | tail -4 | head -2 || exit 1
done
