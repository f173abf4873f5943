#!/bin/bash
# GPU-box check: parity tests, bench (brick + generic), rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first crash/timeout.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
ok_or_fail() { # pytest: 0 pass, 1 test failure (both fine to continue); anything else: stop
  [ "$1" -eq 0 ] || [ "$1" -eq 1 ]
}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
  ok_or_fail $rc || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_brick.log 2>&1 || exit $?
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --path generic > gpurun_out/bench_generic.log 2>&1 || exit $?
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_brick -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_brick.log 2>&1 || exit $?
fi
if [ "$STEP" = dist ]; then
  # N>1 bench flow rehearsal: 2 ranks on the box's single GPU, host-callback communicator
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --comm host --cg-iters 20 > gpurun_out/bench_dist.log 2>&1 || exit $?
fi
if [ "$STEP" = cpu ]; then
  timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1 || exit $?
fi
exit 0
