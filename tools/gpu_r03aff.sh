#!/bin/bash
# round 3: affine-factor brick apply — parity tests, in-process A/B, default bench line
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03aff
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "brick" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python tools/ab_affine.py > $OUT/ab_affine.json 2> $OUT/ab_affine.err || { tail $OUT/ab_affine.err; exit 1; }
cat $OUT/ab_affine.json
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
