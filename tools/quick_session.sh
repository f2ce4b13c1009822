#!/bin/bash
# Iteration session on the GPU box: optional GPU tests (TESTS= pytest selection, "none" to skip), then
# bench.py per workload (WLS) without the CPU leg and the anchor.  Each step under its own time limit;
# a crash or timeout ends the session.  Nothing is built here (build on the CPU host first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/quick_tests.log 2>&1
  rc=$?; echo "== tests rc=$rc"; tail -n 15 gpurun_out/quick_tests.log
  [ $rc -gt 1 ] && exit $rc
fi
for wl in ${WLS:-c2_s1024 c4_teapot}; do
  timeout -k 10 300 python bench.py --workload "$wl" --steps "${STEPS:-20}" --warmup 3 --no-cpu-baseline --no-anchor \
    > "gpurun_out/quick_bench_$wl.log" 2>&1 || { echo "bench $wl failed"; tail -5 "gpurun_out/quick_bench_$wl.log"; exit 1; }
  python - "$wl" <<'PY'
import json, sys
wl = sys.argv[1]
line = [l for l in open(f"gpurun_out/quick_bench_{wl}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"{wl}: {d['ms_per_step']} ms/frame, {d['value']} M samples/s, kernels {d['kernels_ms_per_step']}, "
      f"frac {d['roofline']['frac']}")
PY
done
