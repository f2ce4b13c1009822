#!/bin/bash
# Inter-kernel gap probe (tools/probes/gap_probe.hip) under rocprofv3, then the bench A/B of abtest/ntout
# (tools/patches/nt_output.patch: nontemporal stores of the averaged image) against the product library.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 $R/tools/probes/gap_probe > $R/gpurun_out/gap_plain.log 2>&1 &&
 timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/gap_kt -o run --output-format csv -- $R/tools/probes/gap_probe \
   > $R/gpurun_out/gap_prof.log 2>&1) || { echo "probe failed"; tail -5 $R/gpurun_out/gap_prof.log; exit 1; }
cat gpurun_out/gap_plain.log
python3 tools/probes/gap_stats.py $(find gpurun_out/gap_kt -name "*kernel_trace.csv")
REPS="1 2 3" WLS="c2_s1024 c3_s1024_reflect c4_teapot c5_area_light" VARIANTS="ntout" STEPS=20 bash tools/ab.sh
