#!/bin/bash
# Round 4, first GPU pass: affine-map parity (brick / generic / tile, forms 2/1/0), the touched
# parity tests, the in-process A/B of the three forms at C2, one bench line.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_affine.py tests/test_gpu_parity.py tests/test_gpu_high_order.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/ab_affine.py --rounds 5 --iters 100 > $O/ab_affine.json 2> $O/ab_affine.err || { echo "ab rc=$?"; tail $O/ab_affine.err; exit 1; }
cat $O/ab_affine.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
cat $O/bench.json
