#!/bin/bash
# round-6 diagnostics: dump the tile costs and cost order of a frame (abtest/dump, tools/patches/dump_tile_cost.patch),
# then A/B the product against $VARIANTS
set -e
mkdir -p gpurun_out
for wl in ${DUMP_WLS:-c1_readme c3_s1024_reflect}; do
  RRAY_EXPERIMENT=1 RRAY_LIB=$PWD/abtest/dump/librray_amd.so RRAY_DUMP_TILE_COST=$PWD/gpurun_out/tc_$wl.bin timeout -k 10 200 python bench.py --no-cpu-baseline --no-anchor --no-cold --workload $wl --steps 10 --warmup 3 > gpurun_out/dump_$wl.log 2>&1
done
WLS="${WLS:-c3_s1024_reflect}" VARIANTS="${VARIANTS:-}" REPS="${REPS:-1 2 3}" STEPS=20 timeout -k 10 500 bash tools/ab.sh
