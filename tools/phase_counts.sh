#!/bin/bash
# Experiment: dynamic instruction counts per kernel phase.  The abtest/phase build (tools/patches/
# phase_exit.patch) returns from the fused shade kernel after phase k (RRAY_PHASE_EXIT=k: 1 camera ray,
# 2 trace walk, 3 prepare + children, 4 pattern + prelit, 5 shadow walks + light sum, 0 whole kernel);
# one rocprofv3 --pmc pass per k gives SQ_INSTS_* per wave, so consecutive differences are per phase.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp RRAY_EXPERIMENT=1 RRAY_LIB=$ROOTDIR/abtest/phase/librray_amd.so
WL=${WL:-c2_s1024}
for k in ${KS:-1 2 3 4 5 0}; do
  OUT=$ROOTDIR/gpurun_out/phase_$WL/k$k
  mkdir -p "$OUT"
  (cd /tmp && RRAY_PHASE_EXIT=$k timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM \
     SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d "$OUT" -o run --output-format csv -- \
     python3 "$ROOTDIR/bench.py" --workload "$WL" --steps 3 --warmup 1 --no-cpu-baseline --no-anchor --no-cold) > "$OUT.log" 2>&1 || {
     echo "k=$k failed"; tail -5 "$OUT.log"; exit 1; }
done
python3 - "$WL" <<'PY'
import csv, collections, glob, os, sys
wl = sys.argv[1]
prev = None
for k in [int(x) for x in os.environ.get("KS", "1 2 3 4 5 0").split()]:
    f = glob.glob(f"gpurun_out/phase_{wl}/k{k}/**/run_counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(collections.Counter)
    for r in csv.DictReader(open(f)):
        if "shade_kernel" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.Counter()
    for c in per.values():
        tot.update(c)
    w = tot["SQ_WAVES"]
    row = {c: tot[c] / w for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS")}
    d = {c: row[c] - (prev[c] if prev else 0) for c in row}
    print(f"k={k}: waves {w:.0f} cumulative " + " ".join(f"{c[9:]}={v:.0f}" for c, v in row.items()) +
          "  | phase " + " ".join(f"{c[9:]}={v:.0f}" for c, v in d.items()))
    prev = row
PY
