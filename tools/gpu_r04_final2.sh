#!/bin/bash
# Round-4 closing record: the whole GPU suite and smoke() on the final code, the C2 profile (bench +
# rocprof kernel stats + PMC traffic) and the C5 line.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r04final2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/suite.log 2>&1 || { echo "suite rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | head -20; exit 1; }
tail -2 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 700 bash tools/profile_round.sh r04g c2 || { echo "profile c2 rc=$?"; exit 1; }
echo "profile c2 done"
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 rc=$?"; tail $O/bench_c5.err; exit 1; }
cut -c1-200 $O/bench_c5.json
