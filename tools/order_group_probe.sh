#!/bin/bash
# C5 / C4 with the cost order over groups of a block's four adjacent tiles (RRAY_ORDER_GROUP=4) against single waves: time A/B and the C5 chain kernel's PMC write / fetch bytes.
set -u
cd "${GRAFT_REPO_ROOT}"
ENVS="|RRAY_ORDER_GROUP=4" WLS="c5_area_light c4_teapot" REPS="1 2 3" STEPS=20 BENCH_ARGS="--no-cold" bash tools/ab_envvars.sh || exit 1
export TMPDIR=/tmp
for e in "" "RRAY_ORDER_GROUP=4"; do
  for c in WRITE_SIZE FETCH_SIZE; do
    (cd /tmp && env $e timeout -k 10 240 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/gpurun_out/og_${e:-base}_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5_area_light --steps 3 --warmup 1 --no-cpu-baseline --no-anchor --no-cold) > gpurun_out/og_$c.log 2>&1 || exit 1
  done
done
