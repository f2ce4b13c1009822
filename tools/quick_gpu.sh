#!/bin/bash
# Short GPU iteration: parity tests, bench (no CPU baseline), optional stamps experiment.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b.log 2>&1 || exit 1
echo bench ok
if [ "${STAMPS:-0}" = 1 ]; then
  RRAY_LIB=$PWD/rray_amd/_exp/stamps/librray_amd.so RRAY_STAMPS=$PWD/gpurun_out/stamps.bin \
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/stamps.log 2>&1 || exit 1
  echo stamps ok
fi
