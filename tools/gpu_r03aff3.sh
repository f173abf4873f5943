#!/bin/bash
# round 3: affine factors in the high-order tile apply — ho tests, C3 profile round, C5 line on one GPU
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03aff3
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_high_order.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/profile_round.sh r03aff c3 || exit $?
cat gpurun_out/prof_r03aff_c3/bench.json
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
