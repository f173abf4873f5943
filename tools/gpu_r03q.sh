#!/bin/bash
# round 3q: mixed 16/32-bit SELL columns (tests), SpMV orders / layouts on the unstructured c4u mesh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03q
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fa.py -q -x --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python tools/ab_c4.py --rounds 3 --iters 60 --variants "auto:delaunay:sell_order=3,rcm_win:delaunay:sell_order=2,rcm_glob:delaunay:sell_order=4,geo_glob:delaunay:sell_order=5,rcm_win_nx:delaunay:sell_order=2+spmv_xcd=0,auto32:delaunay:sell_order=3+spmv_index16=0" > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -E '^# |^ "|spmv_us|orth_us|spmv_GBs' $OUT/ab.txt
