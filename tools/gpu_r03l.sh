#!/bin/bash
# round 3l: full GPU suite, smoke, default bench line
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT_TAG:-r03l}
mkdir -p $OUT
T=900 bash tools/gpu_suite.sh; rc=$?
cp gpurun_out/suite.log $OUT/suite.log
tail -3 $OUT/suite.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
