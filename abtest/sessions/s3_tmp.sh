set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1; echo "tests rc=$?"; tail -4 gpurun_out/t3.log
BENCH_ARGS="--workload c3_s1024_reflect --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "c3p4||" "c3p1||RRAY_AA_PASSES=1" "c3p2||RRAY_AA_PASSES=2" "c3p8||RRAY_AA_PASSES=8" "c3nochain||RRAY_NO_CHAIN=1;RRAY_AA_PASSES=1" 2>&1 | cut -c1-250
BENCH_ARGS="--workload c5_area_light --steps 10 --warmup 3 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "c5||" 2>&1 | cut -c1-250
BENCH_ARGS="--workload c2_s1024 --steps 30 --warmup 5 --no-cpu-baseline --no-anchor --no-cold" bash tools/ab_bench.sh "c2||" 2>&1 | cut -c1-250
BENCH_ARGS="--workload c4_teapot --steps 30 --warmup 5 --no-cpu-baseline --no-anchor" bash tools/ab_bench.sh "c4||" 2>&1 | cut -c1-250
grep -o '"cold_frames": \[[^]]*\]' gpurun_out/ab_c4.log | head -2
