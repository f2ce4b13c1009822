#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (each step under its own time limit).
# A step that crashes / times out (exit >= 2 other than pytest's "tests failed" = 1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step build 300 python -c "import __graft_entry__ as g; g.build()" || exit 1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gpu_tests 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python bench.py --steps "$STEPS" --warmup 2 || exit 1
