#!/bin/bash
# Iteration session: GPU parity tests, then every workload benched (no CPU leg) + a one-line summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread \
    ${TESTK:+-k "$TESTK"} > gpurun_out/t.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -3 gpurun_out/t.log
  [ $rc -ne 0 ] && exit $rc
fi
for wl in ${WLS:-c1_readme c2_s1024 c3_s1024_reflect c4_teapot c5_area_light}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-anchor --workload $wl --steps ${STEPS:-20} --warmup ${WARM:-5} \
    ${BENCH_ARGS:-} > gpurun_out/wl_$wl.log 2>&1 || { echo "$wl failed"; tail -5 gpurun_out/wl_$wl.log; exit 1; }
done
python tools/wl_summary.py
