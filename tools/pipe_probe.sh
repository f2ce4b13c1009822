#!/bin/bash
# Frames in flight on one GPU: tools/part_scaling.py pipe (torch streams, k = 2 contexts) for C3 and C2, then
# bench.py with one and two frames in flight.  Each step under its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pipe
for wl in c3_s1024_reflect c2_s1024; do
  timeout -k 10 300 python tools/part_scaling.py $wl 5 pipe > gpurun_out/pipe/ps_$wl.json 2> gpurun_out/pipe/ps_$wl.err \
    || { tail -5 gpurun_out/pipe/ps_$wl.err; exit 1; }
  cat gpurun_out/pipe/ps_$wl.json
done
for wl in c3_s1024_reflect c2_s1024; do
  for f in 1 2; do
    timeout -k 10 300 python bench.py --workload $wl --in-flight $f --no-cold --no-cpu-baseline --no-anchor \
      > gpurun_out/pipe/b_${wl}_$f.log 2>&1 || { tail -5 gpurun_out/pipe/b_${wl}_$f.log; exit 1; }
    echo -n "in-flight $f "; python tools/wl_summary.py gpurun_out/pipe/b_${wl}_$f.log
  done
done
