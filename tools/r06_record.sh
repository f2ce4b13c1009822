#!/bin/bash
# Round-6 record at head, in two GPU calls (each within gpurun's 20-minute limit):
#   PHASE=final  tools/final_session.sh (GPU suite with every full-frame parity test's numbers, smoke, the default
#                bench line and its rocprofv3 kernel trace)
#   PHASE=prof   per-workload kernel trace + PMC passes for C1..C5 (tools/profile_all.sh) and the C3 partition timings
#                (tools/part_scaling.py: bands, and the interleaved parts with rank 0's transfer work)
# Each step has its own limit; the first failure ends the call.  Export afterwards on the host:
#   python tools/export_profiles.py r06 c1_readme c2_s1024 c3_s1024_reflect c4_teapot c5_area_light
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
case "${PHASE:-final}" in
  final)
    bash tools/final_session.sh || exit 1;;
  prof)
    WLS="c1_readme c2_s1024 c3_s1024_reflect c4_teapot c5_area_light" bash tools/profile_all.sh || exit 1
    echo "== part scaling ($(date +%T))"
    timeout -k 10 300 python tools/part_scaling.py c3_s1024_reflect 10 bands > gpurun_out/part_scaling_c3.json \
      2> gpurun_out/part_scaling_c3.err || { tail -5 gpurun_out/part_scaling_c3.err; exit 1; }
    timeout -k 10 300 python tools/part_scaling.py c3_s1024_reflect 10 root > gpurun_out/part_scaling_c3_interleave.json \
      2> gpurun_out/part_scaling_c3_interleave.err || { tail -5 gpurun_out/part_scaling_c3_interleave.err; exit 1; }
    tail -c 400 gpurun_out/part_scaling_c3.json;;
esac
