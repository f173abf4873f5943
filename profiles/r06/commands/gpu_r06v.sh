set -u
# pa_uniform (the common element matrix on the matrix cores): parity, then a C2 A/B against the Kronecker form
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_uniform.py tests/test_gpu_brick_cg.py tests/test_gpu_full_size.py tests/test_gpu_affine.py \
  --durations=10 > $O/tests.log 2>&1 || exit $?
VARIANTS="pa_uniform=1 pa_uniform=0" ROUNDS=2 bash tools/ab_bench.sh $O/ab > $O/ab.log 2>&1 || exit $?
