#!/bin/bash
# Round-6 closing check: the whole GPU suite, smoke(), and the bench lines of C2 (default), C3, C4 and C5
# (one GPU), each from the committed tree.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-closing}; mkdir -p $O
# heartbeat: the suite's longest tests (the full-size oracle checks) print nothing for a minute or two
( while true; do date +%T >> $O/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider --durations=15 > $O/suite.log 2>&1 || { echo "suite rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | head -20; exit 1; }
tail -2 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench rc=$?"; tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 rc=$?"; tail $O/bench_c3.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { echo "c4 rc=$?"; tail $O/bench_c4.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 rc=$?"; tail $O/bench_c5.err; exit 1; }
for f in bench_c2 bench_c3 bench_c4 bench_c5; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$f', '%.4e'%d['value'], d['ms_per_step'], r['bound'], r['frac'], r['avg_launch_us'], r.get('other_kernels_avg_us'), (d.get('gmres') or {}).get('value'))"; done
