#!/bin/bash
# The round's record at head in one GPU call: tools/final_session.sh (GPU suite, smoke, bench line, rocprofv3
# kernel trace of the bench command), then tools/profile_all.sh (per-workload kernel trace + PMC passes).  Export
# the profiles afterwards on the host: python tools/export_profiles.py <tag>.  The first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/final_session.sh || exit 1
bash tools/profile_all.sh || exit 1
