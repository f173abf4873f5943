#!/bin/bash
# Run a subset of the GPU tests (args: pytest selectors) with a time limit; log under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 ${T:-600} python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu "$@" > gpurun_out/subset.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/subset.log; exit $rc
