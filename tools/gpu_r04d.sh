#!/bin/bash
# persistent brick CG A/B + SQ counters of the default C2 bench
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04d}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_brick_cg.py tests/test_gpu_affine.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "brick or xfold" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/ab_opts.py --variant "brick_cg_persist=0" --variant "brick_cg_persist=1" --rounds 5 --iters 100 > $O/ab_opts.json 2> $O/ab_opts.err || { echo "ab rc=$?"; tail $O/ab_opts.err; exit 1; }
cat $O/ab_opts.json
bash tools/pmc_sq.sh $O/sq
python3 tools/pmc_sq_summary.py $O/sq k_brick_cg > $O/sq_summary.json
cat $O/sq_summary.json
