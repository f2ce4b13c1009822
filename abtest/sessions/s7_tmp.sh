set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "chain or mirror" > gpurun_out/t7.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/t7.log
timeout -k 10 600 python tools/part_scaling.py c3_s1024_reflect 5 > gpurun_out/part_scaling_c3.json 2> gpurun_out/part_scaling_c3.err; echo "ps rc=$?"; cat gpurun_out/part_scaling_c3.json
