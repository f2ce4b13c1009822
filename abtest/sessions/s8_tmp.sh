set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t8.log 2>&1; echo "tests rc=$?"; tail -4 gpurun_out/t8.log
BENCH_ARGS="--workload c3_s1024_reflect --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "c3||" "c3nopw||RRAY_NO_PW=1" 2>&1 | cut -c1-250
timeout -k 10 600 python tools/part_scaling.py c3_s1024_reflect 5 > gpurun_out/part_scaling_c3.json 2> gpurun_out/part_scaling_c3.err; echo "ps rc=$?"; cat gpurun_out/part_scaling_c3.json
