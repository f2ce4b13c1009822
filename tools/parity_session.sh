#!/bin/bash
# Full-resolution banded parity + CPU baseline for every BASELINE config on the GPU box:
# bench.py --workload W with its CPU leg (oracle on the box's cores over a band sample, compared with
# the GPU frame row for row).  One step per workload under its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WLS:-c1_readme c4_teapot c5_area_light c3_s1024_reflect}; do
  echo "== $wl ($(date +%T))"
  timeout -k 10 ${T:-600} python bench.py --workload "$wl" --steps ${STEPS:-5} --warmup 2 --no-anchor \
    > "gpurun_out/parity_$wl.log" 2>&1 || { echo "$wl failed rc=$?"; tail -5 "gpurun_out/parity_$wl.log"; exit 1; }
  python - "$wl" <<'PY'
import json, sys
for l in open(f"gpurun_out/parity_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "cpu", d["cpu_baseline"]["value"],
              "parity", d["parity_sample"])
PY
done
