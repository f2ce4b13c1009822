#!/bin/bash
# Round-4 measurements on the GPU box: per-part render times of the C3 partition (one render context per part,
# tools/part_scaling.py), the torus parity tests with their printed bit-exact fractions, then banded full-size
# parity for C3 / C4 / C5 (tools/parity_session.sh).  Each step under its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
timeout -k 10 300 python tools/part_scaling.py c3_s1024_reflect 5 > gpurun_out/r04/part_scaling_c3.json \
  2> gpurun_out/r04/part_scaling_c3.err || { tail -5 gpurun_out/r04/part_scaling_c3.err; exit 1; }
cat gpurun_out/r04/part_scaling_c3.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "torus" > gpurun_out/r04/torus_tests.log 2>&1 || { tail -20 gpurun_out/r04/torus_tests.log; exit 1; }
grep -E "torus|passed|failed" gpurun_out/r04/torus_tests.log | tail -12
WLS="${WLS:-c3_s1024_reflect c4_teapot c5_area_light}" bash tools/parity_session.sh || exit 1
mv gpurun_out/parity_*.log gpurun_out/r04/
