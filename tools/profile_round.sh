#!/bin/bash
# Round profile: bench line (with CPU baseline), rocprofv3 kernel stats of the same bench command,
# PMC HBM traffic passes (FETCH_SIZE, WRITE_SIZE) with stream-probe calibration.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 900 python bench.py --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/stats -o run --output-format csv -- python3 bench.py $ARGS --no-profile-events > $OUT/stats.log 2>&1 || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -T -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cg-iters 20 --no-cpu-baseline --no-profile-events > $OUT/pmc_$C.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -T -d $OUT/calib_$C -o run --output-format csv -- python3 tools/calib.py > $OUT/calib_$C.log 2>&1 || exit $?
done
exit 0
