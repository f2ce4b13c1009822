#!/bin/bash
# Multi-part checks on one GPU: the group tests, the one-rank RCCL tiles path on C3, and tools/part_scaling.py
# (per-part and frame-pipelined render times).  Each step under its own limit; the first failure ends it.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mb
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/mb/tests.log 2>&1 || { tail -30 gpurun_out/mb/tests.log; exit 1; }
tail -1 gpurun_out/mb/tests.log
timeout -k 10 280 python bench.py --force-dist --mode tiles --workload c3_s1024_reflect --steps 10 --warmup 3 --no-cpu-baseline --no-anchor > gpurun_out/mb/tiles_c3.log 2>&1 || { tail -5 gpurun_out/mb/tiles_c3.log; exit 1; }
tail -1 gpurun_out/mb/tiles_c3.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print({k: d[k] for k in ('ms_per_step','single_gpu','speedup_vs_single_gpu','kernels_ms_per_step','tile_identity')})"
timeout -k 10 300 python tools/part_scaling.py c3_s1024_reflect 5 pipe > gpurun_out/mb/pipe.json 2> gpurun_out/mb/pipe.err || { tail -5 gpurun_out/mb/pipe.err; exit 1; }
cat gpurun_out/mb/pipe.json
timeout -k 10 300 python tools/part_scaling.py c2_s1024 50 pipe > gpurun_out/mb/pipe_c2.json 2> gpurun_out/mb/pipe_c2.err || { tail -5 gpurun_out/mb/pipe_c2.err; exit 1; }
cat gpurun_out/mb/pipe_c2.json
