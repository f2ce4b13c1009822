#!/bin/bash
# A/B on the GPU box: the product library and abtest/<variant> builds, interleaved per workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in ${REPS:-1 2}; do
  for wl in ${WLS:-c3_s1024_reflect c5_area_light}; do
    for v in main ${VARIANTS:-}; do
      lib=""; [ "$v" != main ] && lib="RRAY_EXPERIMENT=1 RRAY_LIB=$PWD/abtest/$v/librray_amd.so"
      env $lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-anchor --no-cold --workload $wl --steps ${STEPS:-10} --warmup 3 \
        > gpurun_out/ab/${v}_${wl}_$rep.log 2>&1 || { echo "$v $wl failed"; tail -3 gpurun_out/ab/${v}_${wl}_$rep.log; exit 1; }
      echo -n "$v rep$rep "; python tools/wl_summary.py gpurun_out/ab/${v}_${wl}_$rep.log
    done
  done
done
