#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04e}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_brick_cg.py tests/test_gpu_affine.py tests/test_gpu_parity.py tests/test_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/ab_opts.py --variant "cg_fused_fin=0" --variant "cg_fused_fin=1" --variant "cg_fused_fin=1,cg_xfold=1" --variant "cg_fused_fin=1,cg_ff_blocks=1024" --variant "cg_fused_fin=1,cg_ff_blocks=4096" --rounds 5 --iters 100 > $O/ab_opts.json 2> $O/ab_opts.err || { echo "ab rc=$?"; tail $O/ab_opts.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_opts.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
