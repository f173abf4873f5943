#!/bin/bash
# round 3: LDS layouts with lanes per row on the Kuhn C4 lattice vs its default global sort
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03z3
mkdir -p $OUT
timeout -k 10 700 python tools/ab_c4.py --rounds 3 --iters 60 --variants "k_auto:natural:sell_order=3,k_m512l2:natural:sell_order=6+sell_window=512+spmv_lds=512+spmv_lpr=2,k_m1024l2:natural:sell_order=6+sell_window=1024+spmv_lds=1024+spmv_lpr=2,k_m256l2:natural:sell_order=6+sell_window=256+spmv_lds=256+spmv_lpr=2,k_auto2:natural:sell_order=3,k_m512l2b:natural:sell_order=6+sell_window=512+spmv_lds=512+spmv_lpr=2,k_auto3:natural:sell_order=3,k_m512l2c:natural:sell_order=6+sell_window=512+spmv_lds=512+spmv_lpr=2" > $OUT/ab_kuhn.txt 2>&1 || { tail -20 $OUT/ab_kuhn.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_kuhn.txt
