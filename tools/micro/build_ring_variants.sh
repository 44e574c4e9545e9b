#!/bin/bash
# Build libccrec variants whose NT GEMM register ring is NT_RING deep (dev A/B; the in-tree
# objects must be current: python -m cubecobrarecommender_amd.build).
# usage: tools/micro/build_ring_variants.sh 3 4  -> tools/micro/lib_ring3.so, lib_ring4.so
set -e
cd "$(dirname "$0")/../.."
for r in "$@"; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I include -I cubecobrarecommender_amd/csrc \
    -DNT_RING=$r -c cubecobrarecommender_amd/csrc/gemm.hip -o /tmp/gemm_r$r.o
  objs=$(ls cubecobrarecommender_amd/build_obj/*.o | grep -v gemm.hip.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/gemm_r$r.o -o tools/micro/lib_ring$r.so
  echo "tools/micro/lib_ring$r.so"
done
