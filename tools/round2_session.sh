set -u
# Round-2 session: gpu_session.sh, the library tile group and the torch gather rehearsed with one rank, then parity_session.sh.
[ "${SKIP_SESSION:-0}" = 1 ] || { SKIP_TESTS=0 STEPS=20 bash tools/gpu_session.sh || exit 1; }
timeout -k 10 300 python bench.py --force-dist --mode tiles --workload c3_s1024_reflect --steps 10 --warmup 2 > gpurun_out/tiles_abi.log 2>&1 || { echo tiles_abi failed; tail -20 gpurun_out/tiles_abi.log; exit 1; }
tail -1 gpurun_out/tiles_abi.log | cut -c1-600
timeout -k 10 300 python bench.py --force-dist --gather torch --mode tiles --workload c3_s1024_reflect --steps 10 --warmup 2 > gpurun_out/tiles_torch.log 2>&1 || { echo tiles_torch failed; tail -20 gpurun_out/tiles_torch.log; exit 1; }
tail -1 gpurun_out/tiles_torch.log | cut -c1-600
bash tools/parity_session.sh
