#!/bin/bash
# Experiment: per-wave phase timers (RR_STAMPS build) for the bench workload's level-0 trace/shadow.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RRAY_LIB=$PWD/rray_amd/_exp/stamps/librray_amd.so
for v in lds glb; do
  if [ $v = glb ]; then export RRAY_GLOBAL_CULLS=1; fi
  RRAY_STAMPS=$PWD/gpurun_out/stamps_$v.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 \
    > gpurun_out/stamps_$v.log 2>&1 || exit 1
done
echo done
