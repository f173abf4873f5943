#!/bin/bash
# Round-4 record: the whole GPU suite and smoke(), then the C2 and C3 profiles (bench + rocprof
# kernel stats + PMC traffic) of the final code.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/suite.log 2>&1 || { echo "suite rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | head -20; exit 1; }
tail -2 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 700 bash tools/profile_round.sh r04f c2 || { echo "profile c2 rc=$?"; exit 1; }
echo "profile c2 done"
timeout -k 10 800 bash tools/profile_round.sh r04f c3 || { echo "profile c3 rc=$?"; exit 1; }
echo "profile c3 done"
