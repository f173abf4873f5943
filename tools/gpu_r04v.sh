#!/bin/bash
# GMRES pass 1 with DPP wave sums (gm_dpp): GMRES parity tests and the in-process A/B at C2.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmres.py tests/test_gpu_parity.py tests/test_reference_inputs.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/ab_gmres.py --rounds 5 --iters 60 --variants "gm_dpp=0,gm_dpp=1" > $O/ab_gmres_dpp.json 2> $O/ab.err || { echo "ab rc=$?"; tail $O/ab.err; exit 1; }
cat $O/ab_gmres_dpp.json | head -40
