#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over tools/ab_c4.py variants:
#   bash tools/pmc_ab.sh TAG "<variants>"
# then: python tools/pmc_ab_summary.py gpurun_out/pmc_ab_TAG
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
V=$2
OUT=gpurun_out/pmc_ab_$TAG
mkdir -p $OUT
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 tools/ab_c4.py --rounds 1 --iters 10 --variants "$V" > $OUT/p$i.log 2>&1 || exit $?
  i=$((i+1))
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -d $OUT/calib -o run --output-format csv -- python3 tools/calib.py > $OUT/calib.log 2>&1 || exit $?
exit 0
