#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (each step under its own time limit).
# Nothing is built here: the in-tree .so files travel with the snapshot (build on the CPU host first).
# A step that crashes / times out (exit >= 2 other than pytest's "tests failed" = 1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-20}
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 120 --timeout-method thread
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python bench.py --steps "$STEPS" --warmup 5 || exit 1
