#!/bin/bash
# round 3w: Morton LDS windows on the Kuhn lattice (C4) against the default global sort
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03w
mkdir -p $OUT
timeout -k 10 600 python tools/ab_c4.py --rounds 3 --iters 60 --variants "k_auto:natural:sell_order=3,k_mort512:natural:sell_order=6+sell_window=512+spmv_lds=512,k_mort1024:natural:sell_order=6+sell_window=1024+spmv_lds=1024,k_mort256:natural:sell_order=6+sell_window=256+spmv_lds=256,k_auto2:natural:sell_order=3,k_mort512b:natural:sell_order=6+sell_window=512+spmv_lds=512" > $OUT/ab_kuhn.txt 2>&1 || { tail -20 $OUT/ab_kuhn.txt; exit 1; }
grep -E '^ "|spmv_us' $OUT/ab_kuhn.txt
