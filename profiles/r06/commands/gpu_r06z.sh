set -u
# two-update x-fold at p <= 2: the bitwise x-fold tests and the suites on the brick CG, then C2 bench lines
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_brick_cg.py tests/test_gpu_uniform.py tests/test_distributed.py tests/test_gpu_full_size.py \
  tests/test_gpu_parity.py --durations=10 > $O/tests.log 2>&1 || exit $?
VARIANTS="cg_xfold=1 cg_xfold=0" ROUNDS=2 bash tools/ab_bench.sh $O/ab > $O/ab.log 2>&1 || exit $?
