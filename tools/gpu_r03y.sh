#!/bin/bash
# round 3y: lanes per row of the LDS-staged layout on the unstructured c4u mesh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fa.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python tools/ab_c4.py --rounds 3 --iters 60 --variants "d_l1:delaunay:sell_order=3,d_l2:delaunay:sell_order=3+spmv_lpr=2,d_l4:delaunay:sell_order=3+spmv_lpr=4,d_l4w1024:delaunay:sell_order=6+sell_window=1024+spmv_lds=1024+spmv_lpr=4,d_l2w1024:delaunay:sell_order=6+sell_window=1024+spmv_lds=1024+spmv_lpr=2,d_l1b:delaunay:sell_order=3" > $OUT/ab_del.txt 2>&1 || { tail -20 $OUT/ab_del.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_del.txt
