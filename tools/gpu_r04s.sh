#!/bin/bash
# Round 4: touched parity tests (brick x-fold default, Kronecker tile block order / store policy,
# distributed), C3 A/B of the tile's block order and store policy, the final C2 profile (bench +
# rocprof stats + PMC traffic, per-point leg left out) and the C4 / C5 bench lines.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_brick_cg.py tests/test_gpu_high_order.py tests/test_distributed.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | head -20; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u tools/ab_opts.py --n 128 --p 4 --iters 30 --rounds 3 --variant "ho_xcd=0" --variant "ho_xcd=1" --variant "ho_ye_nt=0" --variant "ho_xcd=1,ho_ye_nt=0" > $O/ab_c3_xcd_nt.json 2> $O/ab_c3.err || { echo "ab rc=$?"; tail $O/ab_c3.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_c3_xcd_nt.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"
timeout -k 10 900 bash tools/profile_round.sh r04 c2 || { echo "profile_round rc=$?"; exit 1; }
echo "profile c2 done"
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 rc=$?"; tail $O/bench_c5.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { echo "c4 rc=$?"; tail $O/bench_c4.err; exit 1; }
for f in bench_c5 bench_c4; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$f', '%.3e'%d['value'], r['bound'], r['frac'], r['avg_launch_us'])"; done
