#!/bin/bash
# Kronecker tile (C3): affected parity tests, in-process A/B at C3 (pa_affine 2 / 1, direction fold),
# C3 bench line.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04k}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_high_order.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u tools/ab_opts.py --n 128 --p 4 --iters 30 --rounds 3 --variant "pa_affine=1" --variant "pa_affine=2,ho_dfold=0" --variant "pa_affine=2,ho_dfold=1" --variant "pa_affine=2,ho_dfold=2" > $O/ab_c3_kron.json 2> $O/ab_c3_kron.err || { echo "ab rc=$?"; tail $O/ab_c3_kron.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_c3_kron.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"
timeout -k 10 500 python -u bench.py --config c3 --steps 3 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench rc=$?"; tail $O/bench_c3.err; exit 1; }
cut -c1-900 $O/bench_c3.json
