#!/bin/bash
# A/B a kernel source change with a probe: builds the probe against the working tree and against
# the original copy in tools/micro/ab_orig/ (same file names), runs both.
# usage: bash tools/micro/ab_probe.sh probe.hip [runs]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
P=$1; N=${2:-1}
mkdir -p tools/micro/bin
F="-O3 -std=c++17 --offload-arch=gfx950 -I include"
hipcc $F -I cubecobrarecommender_amd/csrc tools/micro/$P cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/new 2>/dev/null || exit 1
hipcc $F -I tools/micro/ab_orig -I cubecobrarecommender_amd/csrc tools/micro/$P cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/bin/orig 2>/dev/null || exit 1
for i in $(seq $N); do
  echo "== orig"; timeout -k 5 60 tools/micro/bin/orig | tail -4 || exit 1
  echo "== new"; timeout -k 5 60 tools/micro/bin/new | tail -4 || exit 1
done
