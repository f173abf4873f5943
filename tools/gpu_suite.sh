#!/bin/bash
# Full GPU test suite (pytest -m gpu) with a time limit; log under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 ${T:-1100} python -u -m pytest tests -m gpu -q --maxfail=25 --timeout 300 --timeout-method thread \
    -p no:cacheprovider "$@" > gpurun_out/suite.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/suite.log; exit $rc
