#!/bin/bash
# Kronecker tile at four waves per SIMD (X aliased into the P buffer): high-order parity tests, C3
# A/B, then the final C3 profile (bench + rocprof stats + PMC traffic) and SQ counters.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_high_order.py tests/test_gpu_affine.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u tools/ab_opts.py --n 128 --p 4 --iters 30 --rounds 3 --variant "ho_ktile_waves=3" --variant "ho_ktile_waves=4" > $O/ab_c3_waves.json 2> $O/ab_c3.err || { echo "ab rc=$?"; tail $O/ab_c3.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_c3_waves.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"
bash tools/gpu_r04_prof.sh c3
