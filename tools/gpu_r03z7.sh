#!/bin/bash
# round 3: LDS window sizes around 768 (Kuhn, 2 lanes per row) and 512-896 (Delaunay, 4 lanes per row)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03z7
mkdir -p $OUT
V=""
for rep in a b; do
  for W in 640 768 896; do
    V="$V,k${W}${rep}:natural:sell_order=6+sell_window=$W+spmv_lds=$W+spmv_lpr=2"
  done
done
timeout -k 10 700 python tools/ab_c4.py --rounds 3 --iters 60 --variants "${V:1}" > $OUT/ab_kuhn.txt 2>&1 || { tail -20 $OUT/ab_kuhn.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_kuhn.txt
V=""
for rep in a b; do
  for W in 512 640 768 896; do
    V="$V,d${W}${rep}:delaunay:sell_order=6+sell_window=$W+spmv_lds=$W+spmv_lpr=4"
  done
done
timeout -k 10 900 python tools/ab_c4.py --rounds 3 --iters 60 --variants "${V:1}" > $OUT/ab_del.txt 2>&1 || { tail -20 $OUT/ab_del.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_del.txt
