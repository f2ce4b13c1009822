#!/bin/bash
# Write/fetch attribution on the GPU box: for the product library and each abtest/<variant> (experiment patches that
# remove one store site), one rocprofv3 PMC pass per counter on workload $WL; prints the dominant kernel's
# FETCH_SIZE / WRITE_SIZE per launch.  usage: VARIANTS="xno_stk xno_cost" WL=c3_s1024_reflect tools/attrib_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
WL=${WL:-c3_s1024_reflect}
export TMPDIR=/tmp
mkdir -p gpurun_out/attrib
for v in main ${VARIANTS:-}; do
  if [ "$v" = main ]; then unset RRAY_EXPERIMENT RRAY_LIB; else export RRAY_EXPERIMENT=1 RRAY_LIB=$ROOTDIR/abtest/$v/librray_amd.so; fi
  for c in ${COUNTERS:-WRITE_SIZE FETCH_SIZE}; do
    out=$ROOTDIR/gpurun_out/attrib/${v}_${WL}_$c
    rm -rf "$out"
    (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $c -d "$out" -o run --output-format csv -- \
        python3 "$ROOTDIR/bench.py" --workload "$WL" --steps 3 --warmup 1 --no-cpu-baseline --no-anchor --no-cold \
        --in-flight 1) > "$out.log" 2>&1 || { echo "$v $c failed"; tail -5 "$out.log"; exit 1; }
    python3 - "$out" "$v" "$c" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = {}
for r in rows:
    k = r["Kernel_Name"]
    if "rr::" not in k:
        continue
    acc.setdefault((k, r["Dispatch_Id"]), 0.0)
    acc[(k, r["Dispatch_Id"])] += float(r["Counter_Value"])
per = {}
for (k, d), v in acc.items():
    per.setdefault(k, []).append(v)
for k, vs in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sys.argv[2]:10s} {sys.argv[3]:11s} {sum(vs) / len(vs) / 1024:10.1f} MiB/launch x{len(vs):3d}  {k[:90]}")
    break
PY
  done
done
