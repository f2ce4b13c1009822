#!/bin/bash
# GPU suite + time A/B against abtest/base + the C5 PMC write / fetch attribution of both libraries, one call.
set -u
cd "$GRAFT_REPO_ROOT"
WLS="c5_area_light c3_s1024_reflect" REPS="1 2 3" bash tools/ab_check.sh || exit 1
VARIANTS="base" WL=c5_area_light bash tools/attrib_session.sh || exit 1
