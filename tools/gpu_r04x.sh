#!/bin/bash
# betanom fold into the brick CG apply (cg_beta_fold): brick / parity / distributed tests and the C2 A/B.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_brick_cg.py tests/test_gpu_parity.py tests/test_distributed.py tests/test_gpu_affine.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/ab_opts.py --variant "cg_beta_fold=0" --variant "cg_beta_fold=1" --rounds 7 --iters 100 > $O/ab_c2_beta_fold.json 2> $O/ab.err || { echo "ab rc=$?"; tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_c2_beta_fold.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"
