#!/bin/bash
# A/B timing of experiment builds on the bench workload: each (LIB, ENV) pair runs bench.py once.
# usage: tools/ab_bench.sh "label|lib|ENV=..;.." ...   (lib relative to the repo root; empty = default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  IFS='|' read -r label lib envs <<< "$spec"
  ( [ -n "$lib" ] && export RRAY_EXPERIMENT=1 RRAY_LIB=$PWD/$lib
    for kv in ${envs//;/ }; do export "$kv"; done
    timeout -k 10 200 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/ab_$label.log 2>&1 ) || { echo "$label failed"; tail -5 gpurun_out/ab_$label.log; exit 1; }
  tail -1 gpurun_out/ab_$label.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$label', d['value'], 'ms/step', d['ms_per_step'], 'serial', (d.get('serial') or {}).get('ms_per_step'), 'kernels', d['kernels_ms_per_step'], 'parity', d.get('parity_sample'))"
done
