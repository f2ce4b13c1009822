#!/bin/bash
# parity tests + C2 bench x2 + all workloads (no CPU baseline), each step under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t.log
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/c2_$i.log 2>&1 || exit 1
done
STEPS=${STEPS:-3} timeout -k 10 600 bash tools/all_workloads.sh
