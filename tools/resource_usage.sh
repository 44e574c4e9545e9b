#!/bin/bash
# Per-kernel VGPR/AGPR/scratch/LDS/occupancy of every HIP source (compiler remarks).
# usage: tools/resource_usage.sh [file.hip ...]
cd "$(dirname "$0")/.."
SRCS=${@:-cubecobrarecommender_amd/csrc/*.hip}
for f in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Icubecobrarecommender_amd/csrc \
    -c "$f" -o /tmp/_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v F="$(basename $f)" '/Function Name:/ {n=$(NF-1)} /VGPRs:/ && !/Spill/ {v=$(NF-1)} /AGPRs:/ {a=$(NF-1)}
       /ScratchSize/ {s=$(NF-1)} /Occupancy/ {o=$(NF-1)} /LDS Size/ {l=$(NF-1); printf "%-12s vgpr %3s agpr %3s scratch %4s lds %6s occ %s  %s\n", F, v, a, s, l, o, substr(n,1,90)}'
done
