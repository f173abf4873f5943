#!/bin/bash
# C4 SpMV limiter probe: counter list, then SQ wait/issue split and TA/TCP busy in separate passes
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c4_probe
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
B="python3 bench.py --config c4 --steps 1 --warmup 0 --gmres-iters 30 --no-cpu-baseline --no-profile-events"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -T -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max --kernel-trace -T -d $OUT/ta -o run --output-format csv -- $B > $OUT/ta.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -T -d $OUT/tcp -o run --output-format csv -- $B > $OUT/tcp.log 2>&1 || exit $?
exit 0
