#!/bin/bash
# brick-kernel rework: affected parity tests + in-process A/B of the forms at C2
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04c}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_brick_cg.py tests/test_gpu_affine.py tests/test_gpu_parity.py tests/test_distributed.py tests/test_gpu_gmres.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/ab_opts.py --variant "cg_xfold=0,brick_cg_waves=2" --variant "cg_xfold=1,brick_cg_waves=2" --variant "cg_xfold=0,brick_cg_waves=3" --variant "cg_xfold=1,brick_cg_waves=3" --rounds 5 --iters 100 > $O/ab_opts.json 2> $O/ab_opts.err || { echo "ab rc=$?"; tail $O/ab_opts.err; exit 1; }
cat $O/ab_opts.json
