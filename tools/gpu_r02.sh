#!/bin/bash
# Round-2 GPU check: selected (or all) gpu tests with a per-test time limit, then the bench line.
# usage: bash tools/gpu_r02.sh "<pytest -k expr or empty>" [bench|nobench]
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=20 \
  -p no:cacheprovider "${KARG[@]}" > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${2:-bench}" = bench ]; then
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
fi
exit $rc
