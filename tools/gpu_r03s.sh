#!/bin/bash
# round 3s: LDS-staged SpMV windows (spmv_lds) and Morton orders, Kuhn C4 and unstructured c4u
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03s
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fa.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "lds or mixed or delaunay or index16 or reordered" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python tools/ab_c4.py --rounds 3 --iters 60 --variants "k_auto:natural:sell_order=3,k_win:natural:sell_order=1,k_lds256:natural:sell_order=1+sell_window=256+spmv_lds=256,k_lds512:natural:sell_order=1+sell_window=512+spmv_lds=512,k_lds1024:natural:sell_order=1+sell_window=1024+spmv_lds=1024,k_lds2048:natural:sell_order=1+sell_window=2048+spmv_lds=2048" > $OUT/ab_kuhn.txt 2>&1 || { tail -20 $OUT/ab_kuhn.txt; exit 1; }
grep -E '^ "|spmv_us|spmv_GBs' $OUT/ab_kuhn.txt
timeout -k 10 900 python tools/ab_c4.py --rounds 3 --iters 60 --variants "d_auto:delaunay:sell_order=3,d_mglob:delaunay:sell_order=7,d_rcm512:delaunay:sell_order=2+sell_window=512+spmv_lds=512,d_rcm1024:delaunay:sell_order=2+sell_window=1024+spmv_lds=1024,d_mort512:delaunay:sell_order=6+sell_window=512+spmv_lds=512,d_mort1024:delaunay:sell_order=6+sell_window=1024+spmv_lds=1024,d_mort256:delaunay:sell_order=6+sell_window=256+spmv_lds=256" > $OUT/ab_del.txt 2>&1 || { tail -20 $OUT/ab_del.txt; exit 1; }
grep -E '^ "|spmv_us|spmv_GBs' $OUT/ab_del.txt
