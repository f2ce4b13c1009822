#!/bin/bash
# One GPU call: the GPU suite, then per-workload kernel trace + PMC for $WLS (tools/profile_all.sh).  Each step has
# its own limit; the first failure ends the session.  Output under gpurun_out/check/ and gpurun_out/prof_<wl>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/check
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/check/gpu_tests.log 2>&1 || { tail -30 gpurun_out/check/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/check/gpu_tests.log
fi
WLS="${WLS:-c3_s1024_reflect c5_area_light}" PASSES="${PASSES:-kt fetch write sq}" bash tools/profile_all.sh || exit 1
