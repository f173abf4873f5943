#!/bin/bash
# round 3p: Delaunay FA parity test and the c4u bench line with its profile
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03p
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fa.py -q -x --timeout 250 --timeout-method thread -p no:cacheprovider -k "delaunay" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/profile_round.sh r03z c4u || exit $?
head -c 1500 gpurun_out/prof_r03z_c4u/bench.json; echo
