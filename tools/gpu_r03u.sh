#!/bin/bash
# round 3u: sort window vs LDS window on the unstructured c4u mesh; the auto default
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03u
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fa.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python tools/ab_c4.py --rounds 3 --iters 60 --variants "d_auto:delaunay:sell_order=3,d_s1024_l512:delaunay:sell_order=6+sell_window=1024+spmv_lds=512,d_s2048_l512:delaunay:sell_order=6+sell_window=2048+spmv_lds=512,d_s4096_l512:delaunay:sell_order=6+sell_window=4096+spmv_lds=512,d_s2048_l1024:delaunay:sell_order=6+sell_window=2048+spmv_lds=1024,d_auto2:delaunay:sell_order=3" > $OUT/ab_del.txt 2>&1 || { tail -20 $OUT/ab_del.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_del.txt
