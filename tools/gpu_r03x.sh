#!/bin/bash
# round 3x: physically contiguous device buffers (malloc_contiguous) vs hipMalloc, C4 contexts
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03x
mkdir -p $OUT
timeout -k 10 600 python tools/ab_c4.py --rounds 3 --iters 60 --variants "a1:natural:malloc_contiguous=0,c1:natural:malloc_contiguous=1,a2:natural:malloc_contiguous=0,c2:natural:malloc_contiguous=1,a3:natural:malloc_contiguous=0,c3:natural:malloc_contiguous=1" > $OUT/ab_kuhn.txt 2>&1 || { tail -20 $OUT/ab_kuhn.txt; exit 1; }
grep -E '^ "|spmv_us|orth_us' $OUT/ab_kuhn.txt
