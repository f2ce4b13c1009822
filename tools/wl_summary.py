"""One line per bench log (gpurun_out/wl_*.log or given files): workload, value, ms/step, kernel split."""
import glob
import json
import sys

files = sys.argv[1:] or sorted(glob.glob("gpurun_out/wl_*.log"))
for f in files:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        rf = d.get("roofline") or {}
        ks = " ".join(f"{k}={v}" for k, v in (d.get("kernels_ms_per_step") or {}).items())
        print(f"{d['config']['workload']:18s} {d['value']:10.1f} M/s  {d['ms_per_step']:8.4f} ms  frac={rf.get('frac')}  "
              f"{ks}  host={d.get('host_enqueue_ms_per_step')}")
