#!/bin/bash
# Frame time of a chain workload against the recursion limit (bench.py --max-depth D): what each further depth of
# the reflection chains costs inside the camera waves.  usage: WL=c3_s1024_reflect DEPTHS="0 1 2 3 5" tools/depth_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/depth
WL=${WL:-c3_s1024_reflect}
for d in ${DEPTHS:-0 1 2 3 4 5}; do
  timeout -k 10 300 python bench.py --workload $WL --max-depth $d --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
    --no-anchor --no-cold > gpurun_out/depth/${WL}_d$d.log 2>&1 || { echo "depth $d failed"; tail -3 gpurun_out/depth/${WL}_d$d.log; exit 1; }
  python3 - "$d" gpurun_out/depth/${WL}_d$d.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        j = json.loads(l)
        st = j["stats_last_step"]
        print(f"max_depth {sys.argv[1]}: {j['ms_per_step']:.4f} ms  rays {st['rays']}  shadow {st['shadow_rays']}")
PY
done
