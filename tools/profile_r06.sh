#!/bin/bash
# Round-6 profile of one bench configuration on one box, in one call:
#   1. the bench line (CPU baseline included): event-bracketed apply averages (full launches and all);
#   2. rocprofv3 --kernel-trace --stats of the same bench command without the informational legs (their
#      launches of the same kernel name would be averaged in), and the apply kernel's per-launch CSV and
#      averages (tools/rocprof_avg.py -> profiles/rocprof_kernels.json) that the bench line quotes.
# usage: bash tools/profile_r06.sh TAG c2|c3|c5 [extra bench args]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
CFG=$2
shift 2
OUT=gpurun_out/${TAG}_${CFG}
mkdir -p $OUT
case $CFG in
  c2) KEY=n64_p2_k7_aff; KERN=k_brick_cg;;
  c3) KEY=n128_p4_k7_aff; KERN=k_hobrick_cg;;
  c5) KEY=n256_p2_k7_aff; KERN=k_brick_cg;;
esac
timeout -k 10 600 python -u bench.py --config $CFG --steps 5 --warmup 1 "$@" > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/stats -o run --output-format csv -- python3 bench.py \
    --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-profile-events --no-kron-form --spd-steps 0 --per-point-steps 0 \
    --gmres-iters 0 "$@" > $OUT/stats.log 2>&1 || exit $?
python3 tools/rocprof_avg.py --trace $OUT/stats --kernel $KERN --key $KEY --csv $OUT/${KERN}_launches.csv \
    --json $OUT/rocprof_kernels.json > $OUT/rocprof_avg.json || exit $?
exit 0
