#!/bin/bash
# rocprofv3 for every GPU workload (C2, C3, C4, C5): kernel trace + stats, then separate PMC passes
# (SQ instruction/wait counters, FETCH_SIZE, WRITE_SIZE), each its own run; then the per-level
# breakdown (tools/profile_levels.py) -> gpurun_out/prof_<wl>/levels.json.  Copy to profiles/ after.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for wl in ${WLS:-c2_s1024 c3_s1024_reflect c4_teapot c5_area_light}; do
  steps=20; [ "$wl" = c2_s1024 ] && steps=50; [ "$wl" = c3_s1024_reflect ] && steps=10
  rm -rf "gpurun_out/prof_$wl"
  WL=$wl SKIP_BUILD=1 STEPS=$steps PASSES="${PASSES:-kt sq fetch write}" PROF_DIR="prof_$wl" \
    bash tools/profile_session.sh > "gpurun_out/prof_$wl.log" 2>&1 || { echo "$wl profile failed"; tail -5 "gpurun_out/prof_$wl.log"; exit 1; }
  echo "== $wl"
  python tools/profile_levels.py "gpurun_out/prof_$wl" "gpurun_out/prof_$wl/levels.json" || exit 1
  python -c "from rray_amd.build import source_digest; print(source_digest())" > "gpurun_out/prof_$wl/src_digest"
done
