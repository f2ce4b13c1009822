#!/bin/bash
# Bench A/B of environment settings on the in-tree library, interleaved per repetition and workload.
# usage: ENVS="|XX_A=1|XX_B=1" WLS="c2_s1024 c4_teapot" REPS="1 2" STEPS=30 tools/ab_envvars.sh
# (ENVS: '|'-separated; an empty entry is the baseline).  Optional TESTS=<pytest selection> first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/ab_tests.log 2>&1; rc=$?
  echo "== tests rc=$rc"; tail -n 6 gpurun_out/ab_tests.log; [ $rc -gt 1 ] && exit $rc
fi
IFS='|' read -r -a envs <<< "${ENVS:-}"
[ ${#envs[@]} -eq 0 ] && envs=("")
for rep in ${REPS:-1 2}; do
  for wl in ${WLS:-c2_s1024}; do
    for e in "${envs[@]}"; do
      env $e timeout -k 10 300 python bench.py --workload "$wl" --steps "${STEPS:-30}" --warmup 5 --no-cpu-baseline \
        --no-anchor ${BENCH_ARGS:-} > gpurun_out/ab_run.log 2>&1 || { echo "bench failed: $wl [$e]"; tail -5 gpurun_out/ab_run.log; exit 1; }
      python - "$wl" "$e" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab_run.log") if l.startswith("{")][-1])
print(f"{sys.argv[1]:18s} [{sys.argv[2] or 'base':24s}] {d['ms_per_step']:8.4f} ms  kernels {d['kernels_ms_per_step']}")
PY
    done
  done
done
