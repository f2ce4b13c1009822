#!/bin/bash
# rocprofv3 session for the bench workload: kernel-trace stats, then one PMC pass per counter group
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  No --sys-trace / runtime trace with --pmc.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out/${PROF_DIR:-prof}
WL=${WL:-c2_s1024}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${SKIP_BUILD:-0}" != 1 ]; then
  python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || exit 1
fi
STEPS=${STEPS:-50}  # the kernel-trace pass runs as many steps as the default bench line (clocks settle)
run() {  # name, timeout, rocprof args...  (PSTEPS: steps of this pass)
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  (cd /tmp && timeout -k 10 "$t" rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- \
      python3 "$ROOTDIR/bench.py" --workload "$WL" --steps "${PSTEPS:-5}" --warmup "${PWARM:-1}" --no-cpu-baseline --no-anchor --no-cold --in-flight 1) > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  return $rc
}
PASSES=${PASSES:-kt fetch write sq sq2}  # subset to run (each pass is its own rocprofv3 run)
for p in $PASSES; do
  case $p in
    kt) PSTEPS=$STEPS PWARM=5 run kt 300 --kernel-trace --stats || exit 1;;
    fetch) run pmc_fetch 300 --pmc FETCH_SIZE || exit 1;;
    write) run pmc_write 300 --pmc WRITE_SIZE || exit 1;;
    sq) run pmc_sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU || exit 1;;
    sq2) run pmc_sq2 300 --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE || exit 1;;
  esac
done
find "$OUT" -name "*.csv" | head -50
