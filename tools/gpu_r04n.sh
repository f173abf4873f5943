#!/bin/bash
# Round 4: high-order (Kronecker tile + direction / x folds) and brick column-walk parity tests,
# in-process A/B at C3 and C2, C3 and C2 bench lines.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04n}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_high_order.py tests/test_gpu_brick_cg.py tests/test_gpu_affine.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/ab_opts.py --variant "brick_cols=0" --variant "brick_cols=1" --variant "brick_cols=1,cg_xfold=1" --rounds 5 --iters 100 > $O/ab_c2_cols.json 2> $O/ab_c2_cols.err || { echo "ab rc=$?"; tail $O/ab_c2_cols.err; exit 1; }
timeout -k 10 500 python -u tools/ab_opts.py --n 128 --p 4 --iters 30 --rounds 3 --variant "ho_dfold=0" --variant "ho_dfold=1" --variant "ho_dfold=2" > $O/ab_c3_dfold.json 2> $O/ab_c3_dfold.err || { echo "ab rc=$?"; tail $O/ab_c3_dfold.err; exit 1; }
for f in ab_c2_cols ab_c3_dfold; do python3 -c "
import json; d=json.load(open('$O/$f.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"; done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
