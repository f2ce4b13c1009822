#!/bin/bash
# Bench every workload once (no CPU baseline) — timing + stats per workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WLS:-c1_readme c2_s1024 c3_s1024_reflect c4_teapot c5_area_light}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-anchor --workload $wl --steps ${STEPS:-3} --warmup 1 \
    > gpurun_out/wl_$wl.log 2>&1 || { echo "$wl failed"; tail -5 gpurun_out/wl_$wl.log; exit 1; }
  echo "$wl ok"
done
