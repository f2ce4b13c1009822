#!/bin/bash
# Parity of a few scenes under experiment builds (abtest/<name>, see build.build_variant),
# each run twice to expose run-to-run differences.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=${K:-'shape_scenes and (glass or mixed or noise_mix)'}
for v in ${VARIANTS:-default}; do
  case $v in
    default) env="RRAY_X=0";;
    unfused) env="RRAY_UNFUSED=1";;
    *) env="RRAY_EXPERIMENT=1 RRAY_LIB=$PWD/abtest/$v/librray_amd.so";;
  esac
  for r in 1 2; do
    echo "== $v run $r"
    env $env timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -k "$K" -s > gpurun_out/diag_${v}_$r.log 2>&1
    rc=$?
    grep -E "max\|d\||passed|failed" gpurun_out/diag_${v}_$r.log | grep -v print
    [ $rc -gt 1 ] && exit $rc
  done
done
exit 0
