#!/bin/bash
# Experiment: where a wave's cycles go, per kernel phase.  For each RRAY_PHASE_EXIT=k of the abtest/phase build
# (tools/patches/phase_exit.patch; see tools/phase_times.sh), one rocprofv3 --pmc pass of SQ wave-cycle counters
# (quad-cycles): parked on s_waitcnt / barriers (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY), issuing
# (SQ_ACTIVE_INST_ANY; VALU / scalar parts).  Consecutive differences attribute them to phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp RRAY_EXPERIMENT=1 RRAY_LIB=$ROOTDIR/abtest/phase/librray_amd.so
for WL in ${WLS:-c4_teapot c2_s1024}; do
  for k in ${KS:-1 14 2 4 24 5 0}; do
    OUT=$ROOTDIR/gpurun_out/phase_pmc_$WL/k$k
    mkdir -p "$OUT"
    (cd /tmp && RRAY_PHASE_EXIT=$k timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
       SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES -d "$OUT" -o run --output-format csv -- \
       python3 "$ROOTDIR/bench.py" --workload "$WL" --steps 3 --warmup 1 --no-cpu-baseline --no-anchor) > "$OUT.log" 2>&1 || {
       echo "$WL k=$k failed"; tail -5 "$OUT.log"; exit 1; }
  done
  python3 - "$WL" <<'PY'
import csv, collections, glob, os, sys
wl = sys.argv[1]
prev = None
names = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA")
for k in [int(x) for x in os.environ.get("KS", "1 14 2 4 24 5 0").split()]:
    f = glob.glob(f"gpurun_out/phase_pmc_{wl}/k{k}/**/run_counter_collection.csv", recursive=True)[0]
    tot = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "shade_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    w = tot["SQ_WAVES"]
    row = {c: 4 * tot[c] / w for c in names}  # cycles per wave
    d = {c: row[c] - (prev[c] if prev else 0) for c in row}
    print(f"{wl} k={k:>2}: per wave " + " ".join(f"{c[3:]}={v:.0f}" for c, v in row.items()) +
          " | phase " + " ".join(f"{c[3:]}={v:.0f}" for c, v in d.items()))
    prev = row
PY
done
