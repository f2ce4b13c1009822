#!/bin/bash
# Experiment: kernel time per phase.  The abtest/phase build (tools/patches/phase_exit.patch) ends the
# fused shade kernel's waves after phase k (RRAY_PHASE_EXIT=k: 1 camera ray, 2 trace walk, 3 prepare +
# children, 4 pattern + prelit, 5 shadow walks + light sum, 0 whole kernel; 11-14 / 21-24 inside the trace /
# shadow walk); the bench's kernel time per k, so consecutive differences are what each phase costs at the
# kernel's occupancy.  Build first: python rray_amd/build.py variant phase --patch tools/patches/phase_exit.patch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/phase_times
export RRAY_EXPERIMENT=1 RRAY_LIB=$PWD/abtest/phase/librray_amd.so
for wl in ${WLS:-c4_teapot c2_s1024}; do
  for k in ${KS:-1 11 12 13 14 2 3 4 21 22 23 24 5 0}; do
    RRAY_PHASE_EXIT=$k timeout -k 10 200 python bench.py --workload "$wl" --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --no-anchor > gpurun_out/phase_times/${wl}_k$k.log 2>&1 || { echo "$wl k=$k failed"; tail -3 gpurun_out/phase_times/${wl}_k$k.log; exit 1; }
    python - "$wl" "$k" <<'PY'
import json, sys
wl, k = sys.argv[1:]
d = json.loads([l for l in open(f"gpurun_out/phase_times/{wl}_k{k}.log") if l.startswith("{")][-1])
print(f"{wl} k={k:>2}: kernel {d['kernels_ms_per_step']}")
PY
  done
done
