#!/bin/bash
# Per-dispatch kernel trace of one frame of a workload (rocprofv3 --kernel-trace): which level /
# kernel the frame's time goes to.  usage: WL=c3_s1024_reflect tools/level_trace.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out/lt_${WL:-c3_s1024_reflect}
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv -- \
    python3 "$ROOTDIR/bench.py" --workload "${WL:-c3_s1024_reflect}" --steps 1 --warmup 1 --no-cpu-baseline) \
    > "$OUT/run.log" 2>&1 || { tail -5 "$OUT/run.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rr" in r["Kernel_Name"]]
half = len(rows) // 2  # warmup frame, then the timed frame
for r in rows[half:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"].split("(")[0].replace("void rr::", "")
    print(f"{name[:60]:60s} grid {int(r['Grid_Size_X']) if 'Grid_Size_X' in r else r.get('Grid_Size','?')}  {d:9.1f} us")
PY
