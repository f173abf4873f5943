#!/bin/bash
# round 3g: kernel timelines (rocprofv3 kernel trace) of the C2 GMRES leg, the C3 CG and the C4
# GMRES, for the idle-gap and per-kernel breakdown (tools/trace_gaps.py)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03g
mkdir -p $OUT
COMMON="--steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --spd-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c2 -o run --output-format csv -- python3 bench.py $COMMON --cg-iters 4 --gmres-iters 60 > $OUT/c2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/c3 -o run --output-format csv -- python3 bench.py --config c3 $COMMON --cg-iters 6 --gmres-iters 0 > $OUT/c3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c4 -o run --output-format csv -- python3 bench.py --config c4 $COMMON --gmres-iters 30 > $OUT/c4.log 2>&1 || exit $?
for C in c2 c3 c4; do
  f=$(ls $OUT/$C/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(ls $OUT/$C/run_kernel_trace.csv)
  cp "$f" $OUT/${C}_kernel_trace.csv
done
echo done
