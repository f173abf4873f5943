#!/bin/bash
# round 3t: LDS window sizes, finer
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03t
mkdir -p $OUT
timeout -k 10 600 python tools/ab_c4.py --rounds 3 --iters 60 --variants "k_auto:natural:sell_order=3,k_lds128:natural:sell_order=1+sell_window=128+spmv_lds=128,k_lds192:natural:sell_order=1+sell_window=192+spmv_lds=192,k_lds256:natural:sell_order=1+sell_window=256+spmv_lds=256,k_lds384:natural:sell_order=1+sell_window=384+spmv_lds=384,k_lds256nx:natural:sell_order=1+sell_window=256+spmv_lds=256+spmv_xcd=0,k_lds256b:natural:sell_order=1+sell_window=256+spmv_lds=256" > $OUT/ab_kuhn.txt 2>&1 || { tail -20 $OUT/ab_kuhn.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_kuhn.txt
timeout -k 10 900 python tools/ab_c4.py --rounds 3 --iters 60 --variants "d_mort256:delaunay:sell_order=6+sell_window=256+spmv_lds=256,d_mort384:delaunay:sell_order=6+sell_window=384+spmv_lds=384,d_mort512:delaunay:sell_order=6+sell_window=512+spmv_lds=512,d_mort768:delaunay:sell_order=6+sell_window=768+spmv_lds=768,d_mort512nx:delaunay:sell_order=6+sell_window=512+spmv_lds=512+spmv_xcd=0,d_mort512b:delaunay:sell_order=6+sell_window=512+spmv_lds=512" > $OUT/ab_del.txt 2>&1 || { tail -20 $OUT/ab_del.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_del.txt
