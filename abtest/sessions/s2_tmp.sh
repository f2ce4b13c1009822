set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "chain or shape or torus or mirror or cost_ordered" > gpurun_out/t2.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/t2.log
BENCH_ARGS="--workload c3_s1024_reflect --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "main||" "nochain||RRAY_NO_CHAIN=1" "rmd3|abtest/chain_rmd3/librray_amd.so|" "rmd4|abtest/chain_rmd4/librray_amd.so|" 2>&1 | cut -c1-300
BENCH_ARGS="--workload c5_area_light --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "c5main||" "c5nochain||RRAY_NO_CHAIN=1" "c5rmd3|abtest/chain_rmd3/librray_amd.so|" 2>&1 | cut -c1-300
BENCH_ARGS="--workload c3_s1024_reflect --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "main_pass1||RRAY_AA_PASSES=1" "main_pass8||RRAY_AA_PASSES=8" 2>&1 | cut -c1-300
