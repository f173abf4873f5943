#!/bin/bash
# den fold with the partial loads in one round trip: brick CG tests and the C2 A/B of the grid size.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_brick_cg.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/ab_opts.py --variant "cg_den_fold=1024" --variant "cg_den_fold=1536" --variant "cg_den_fold=2048" --variant "cg_den_fold=3072" --rounds 7 --iters 100 > $O/ab_c2_den_fold3.json 2> $O/ab.err || { echo "ab rc=$?"; tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_c2_den_fold3.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"
