#!/bin/bash
# Round-5 record at head in one GPU call: tools/round_record.sh (GPU suite, smoke, default bench line + its kernel
# trace, per-workload kernel trace + PMC), full-frame banded parity for C3 / C4 / C5 (C5 at --cpu-stride 4: 270 rows),
# and the C3 partition timings (tools/part_scaling.py).  Each step has its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/round_record.sh || exit 1
mkdir -p gpurun_out/parity
for spec in "c3_s1024_reflect" "c4_teapot" "c5_area_light --cpu-stride 4"; do
  wl=${spec%% *}
  echo "== parity $spec ($(date +%T))"
  timeout -k 10 600 python bench.py --workload $spec --steps 5 --warmup 2 --no-anchor \
    > "gpurun_out/parity/parity_$wl.log" 2>&1 || { echo "$wl failed"; tail -5 "gpurun_out/parity/parity_$wl.log"; exit 1; }
  grep -o '"parity_sample": {[^}]*}' "gpurun_out/parity/parity_$wl.log"
done
echo "== part scaling ($(date +%T))"
timeout -k 10 600 python tools/part_scaling.py c3_s1024_reflect 5 > gpurun_out/part_scaling_c3.json 2> gpurun_out/part_scaling_c3.err \
  || { tail -5 gpurun_out/part_scaling_c3.err; exit 1; }
tail -c 600 gpurun_out/part_scaling_c3.json
