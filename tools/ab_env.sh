#!/bin/bash
# GPU parity tests, then bench A/B of the in-tree library against abtest/<variant> builds, interleaved
# per workload and repetition.  usage: VARIANTS="base" WLS="c2_s1024 c3_s1024_reflect" REPS="1 2" tools/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
tail -2 gpurun_out/t.log; [ $rc -gt 1 ] && exit $rc
exec_ab() { REPS="${REPS:-1 2}" WLS="${WLS:-c2_s1024}" VARIANTS="${VARIANTS:-base}" STEPS=${STEPS:-20} bash tools/ab.sh; }
exec_ab
