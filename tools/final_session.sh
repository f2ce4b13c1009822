#!/bin/bash
# End-of-round record on the GPU box: parity suite, smoke, the default bench line, and a rocprofv3
# kernel trace (--kernel-trace --stats) of that same bench command.  Each step has its own limit; the
# first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/final/gpu_tests.log 2>&1 || { tail -20 gpurun_out/final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2>&1 || exit 1
tail -1 gpurun_out/final/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final/kt -o kt --output-format csv -- \
  python bench.py --no-cpu-baseline > gpurun_out/final/kt.log 2>&1 || exit 1
find gpurun_out/final/kt -name "*kernel_stats.csv" | head -3
