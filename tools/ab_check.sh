#!/bin/bash
# GPU suite at the working tree's build, then bench A/B against abtest/<variant> builds (tools/ab.sh), in one call.
# usage: VARIANTS="base" WLS="c5_area_light" REPS="1 2 3" tools/ab_check.sh   (SKIP_TESTS=1 skips the suite)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/check
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  RRAY_TRACE_FILE=$PWD/gpurun_out/check/trace.log timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/check/gpu_tests.log 2>&1 || { tail -30 gpurun_out/check/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/check/gpu_tests.log
fi
REPS="${REPS:-1 2 3}" WLS="${WLS:-c5_area_light}" VARIANTS="${VARIANTS:-base}" STEPS=${STEPS:-20} bash tools/ab.sh
