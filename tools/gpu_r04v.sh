#!/bin/bash
# GMRES pass 1 with DPP wave sums (gm_dpp) and the structured Mult through the patch buffer
# (brick_mult_pb): GMRES / brick parity tests and the in-process A/B of the C2 GMRES(30) leg.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gmres.py tests/test_gpu_parity.py tests/test_reference_inputs.py tests/test_gpu_brick_cg.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/ab_gmres.py --rounds 5 --iters 60 --variants "gm_dpp=0/brick_mult_pb=0,gm_dpp=1/brick_mult_pb=0,gm_dpp=1/brick_mult_pb=1" > $O/ab_gmres.json 2> $O/ab.err || { echo "ab rc=$?"; tail $O/ab.err; exit 1; }
cat $O/ab_gmres.json | head -60
