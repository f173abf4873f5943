#!/bin/bash
# round 3k: small-problem GMRES latency (tools/small_solve.py) and its kernel timeline
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03k
mkdir -p $OUT
timeout -k 10 300 python tools/small_solve.py --iters 300 --rounds 3 > $OUT/small.txt 2>&1 || { tail -20 $OUT/small.txt; exit 1; }
grep -v "^ " $OUT/small.txt | head -8
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 tools/small_solve.py --iters 120 --rounds 1 --problems square,q64 > $OUT/tr.log 2>&1 || exit $?
f=$(ls $OUT/tr/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$OUT/tr/run_kernel_trace.csv
cp "$f" $OUT/kernel_trace.csv
python tools/trace_gaps.py $OUT/kernel_trace.csv --after k_gm_init | head -30
