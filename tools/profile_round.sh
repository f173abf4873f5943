#!/bin/bash
# Round profile of one bench configuration:
#   bench line (with CPU baseline), rocprofv3 kernel stats of the same bench command, and
#   PMC HBM traffic passes (FETCH_SIZE, WRITE_SIZE) plus the stream-probe calibration pass.
#   The rocprof passes leave out the bench's per-point-stream leg (a second context whose apply is the
#   same kernel with the per-point data) and the GMRES leg (at p >= 3 its Mult is the same tile kernel):
#   their launches would be averaged into the timed kernel.
# usage: bash tools/profile_round.sh TAG [c2|c3|c4|c4s|c4u]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
CFG=${2:-c2}
OUT=gpurun_out/prof_${TAG}_${CFG}
mkdir -p $OUT
case $CFG in
  c2) SHORT="--cg-iters 20 --spd-steps 0";;
  c3) SHORT="--cg-iters 4 --gmres-iters 0 --spd-steps 0";;
  c4|c4s|c4u) SHORT="--gmres-iters 30";;
  c5) SHORT="--cg-iters 10 --gmres-iters 0 --spd-steps 0";;
esac
timeout -k 10 900 python bench.py --config $CFG --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/stats -o run --output-format csv -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-profile-events --no-kron-form --spd-steps 0 --per-point-steps 0 --gmres-iters 0 > $OUT/stats.log 2>&1 || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -T -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --config $CFG --steps 1 --warmup 0 $SHORT --no-cpu-baseline --no-profile-events --no-kron-form --per-point-steps 0 > $OUT/pmc_$C.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -T -d $OUT/calib_$C -o run --output-format csv -- python3 tools/calib.py > $OUT/calib_$C.log 2>&1 || exit $?
done
exit 0
