#!/bin/bash
# round 3r: Morton SpMV orders and window sizes on the unstructured c4u mesh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03r
mkdir -p $OUT
timeout -k 10 1000 python tools/ab_c4.py --rounds 3 --iters 60 --variants "auto:delaunay:sell_order=3,mort_glob:delaunay:sell_order=7,mort_w256:delaunay:sell_order=6+sell_window=256,mort_w1024:delaunay:sell_order=6+sell_window=1024,mort_w4096:delaunay:sell_order=6+sell_window=4096,rcm_w512:delaunay:sell_order=2+sell_window=512,rcm_w128:delaunay:sell_order=2+sell_window=128" > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -E '^# |^ "|spmv_us|spmv_GBs' $OUT/ab.txt
