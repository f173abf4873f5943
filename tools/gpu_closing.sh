#!/bin/bash
# Closing check of a round: the whole GPU suite, smoke(), the default
# bench line and the C3 line (C4=1: and the C4 line).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-closing}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/suite.log 2>&1 || { echo "suite rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | head -20; exit 1; }
tail -2 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench rc=$?"; tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 rc=$?"; tail $O/bench_c3.err; exit 1; }
if [ -n "${C4:-}" ]; then
  timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { echo "c4 rc=$?"; tail $O/bench_c4.err; exit 1; }
fi
for f in bench_c2 bench_c3 ${C4:+bench_c4}; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$f', '%.4e'%d['value'], r['bound'], r['frac'], r['avg_launch_us'], r['other_kernels_avg_us'])"; done
