#!/bin/bash
# round 3i: den-only grid ticket (grid_fin) A/B on the C2 CG; chunked SELL layouts (spmv_chunk) on C4
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fa.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/fa_tests.log 2>&1 || { tail -30 $OUT/fa_tests.log; exit 1; }
tail -2 $OUT/fa_tests.log
timeout -k 10 300 python tools/ab.py --no-events --rounds 6 --variants grid_fin=0,grid_fin=1 > $OUT/ab_cg.txt 2>&1 || exit $?
tail -16 $OUT/ab_cg.txt
timeout -k 10 400 python tools/ab_c4.py --rounds 6 --variants "g1:natural:spmv_chunk=1,g2:natural:spmv_chunk=2,g4:natural:spmv_chunk=4,w1:natural:sell_order=1,w2:natural:sell_order=1+spmv_chunk=2,w4:natural:sell_order=1+spmv_chunk=4,g1b:natural:spmv_chunk=1,g2b:natural:spmv_chunk=2" > $OUT/ab_c4.txt 2>&1 || exit $?
grep -E '^ "|spmv_us|orth_us' $OUT/ab_c4.txt
