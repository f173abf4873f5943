#!/bin/bash
# round 3: window size of the LDS default on the Kuhn C4 lattice (2 lanes per row), two contexts each
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03z6
mkdir -p $OUT
V=""
for rep in a b; do
  for W in 384 512 768 1024; do
    V="$V,w${W}${rep}:natural:sell_order=6+sell_window=$W+spmv_lds=$W+spmv_lpr=2"
  done
done
timeout -k 10 900 python tools/ab_c4.py --rounds 3 --iters 60 --variants "${V:1}" > $OUT/ab_kuhn.txt 2>&1 || { tail -20 $OUT/ab_kuhn.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_kuhn.txt
