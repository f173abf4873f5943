#!/bin/bash
# Round-4 record, part 1: the whole GPU suite and smoke() (logs under gpurun_out/$TAG).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04f}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/suite.log 2>&1 || { echo "suite rc=$?"; tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
