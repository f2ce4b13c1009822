#!/bin/bash
# bench.py (no CPU baseline) under experiment builds (abtest/<name>, build.build_variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  case $v in
    default) env="RRAY_X=0";;
    *) env="RRAY_EXPERIMENT=1 RRAY_LIB=$PWD/abtest/$v/librray_amd.so";;
  esac
  env $env timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bv_$v.log 2>&1 || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bv_$v.log').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
