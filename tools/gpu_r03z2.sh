#!/bin/bash
# round 3 final profiles, part 2: C3 and C4
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/profile_round.sh r03z c3 || exit $?
bash tools/profile_round.sh r03z c4 || exit $?
head -c 400 gpurun_out/prof_r03z_c3/bench.json; echo; head -c 400 gpurun_out/prof_r03z_c4/bench.json; echo
