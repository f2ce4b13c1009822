set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in 0 1 2 3 4 5; do
timeout -k 10 300 python bench.py --workload c3_s1024_reflect --steps 8 --warmup 2 --no-cpu-baseline --no-anchor --no-cold --max-depth $d > gpurun_out/d$d.log 2>&1 || exit 1
python - $d <<'PY'
import json,sys
d=json.loads([l for l in open(f"gpurun_out/d{sys.argv[1]}.log") if l.startswith("{")][-1])
print("depth", sys.argv[1], d["ms_per_step"], d["kernels_ms_per_step"], {k: d["stats_last_step"][k] for k in ("rays","shadow_rays","shade_events")})
PY
done
