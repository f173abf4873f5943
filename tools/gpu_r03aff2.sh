#!/bin/bash
# round 3: affine-factor brick apply — C2 profile round (bench, rocprof stats, PMC), then the full GPU suite
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/profile_round.sh r03aff c2 || exit $?
cat gpurun_out/prof_r03aff_c2/bench.json
T=900 bash tools/gpu_suite.sh; rc=$?
mkdir -p gpurun_out/r03aff2; cp gpurun_out/suite.log gpurun_out/r03aff2/suite.log
tail -3 gpurun_out/r03aff2/suite.log
exit $rc
