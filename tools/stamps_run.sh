#!/bin/bash
# Experiment: per-wave phase timers for the bench workload's level-0 kernel.  Build the variant first:
#   python rray_amd/build.py variant stamps --patch tools/patches/stamps.patch RR_STAMPS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RRAY_EXPERIMENT=1 RRAY_LIB=$PWD/abtest/stamps/librray_amd.so
RRAY_STAMPS=$PWD/gpurun_out/stamps.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 \
  ${BENCH_ARGS:-} > gpurun_out/stamps.log 2>&1 || exit 1
python tools/stamps_summary.py gpurun_out/stamps.bin
