#!/bin/bash
# round 3: full GPU suite with the LDS default, then the C4 profile
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03z4
mkdir -p $OUT
T=800 bash tools/gpu_suite.sh; rc=$?
cp gpurun_out/suite.log $OUT/suite.log
tail -3 $OUT/suite.log
[ $rc -le 1 ] || exit $rc
bash tools/profile_round.sh r03x c4 || exit $?
head -c 1200 gpurun_out/prof_r03x_c4/bench.json
