#!/bin/bash
# round 3j: chunked SELL (spmv_chunk) on the windowed vs global layouts, three contexts each, C4
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fa.py tests/test_gpu_gmres.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 500 python tools/ab_c4.py --rounds 6 --variants "g1a:natural:spmv_chunk=1,w2a:natural:sell_order=1+spmv_chunk=2,g1b:natural:spmv_chunk=1,w2b:natural:sell_order=1+spmv_chunk=2,g1c:natural:spmv_chunk=1,w2c:natural:sell_order=1+spmv_chunk=2,w2u8:natural:sell_order=1+spmv_chunk=2+spmv_u=8,g2u8:natural:spmv_chunk=2+spmv_u=8,w2nx:natural:sell_order=1+spmv_chunk=2+spmv_xcd=0,s2:shuffled:sell_order=2+spmv_chunk=2" > $OUT/ab_c4.txt 2>&1 || exit $?
grep -E '^ "|spmv_us|orth_us' $OUT/ab_c4.txt
