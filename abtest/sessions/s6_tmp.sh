set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "chain or mirror or render_matches" > gpurun_out/t6.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/t6.log
BENCH_ARGS="--workload c3_s1024_reflect --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "c3||" "c3nodeep||RRAY_NO_DEEP=1" 2>&1 | cut -c1-250
