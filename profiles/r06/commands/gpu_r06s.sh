set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_partition.py tests/test_gpu_gmres.py "tests/test_distributed.py::test_gpu_gmres_two_ranks_one_device" \
  "tests/test_distributed.py::test_gpu_high_order_two_ranks_one_device" --durations=10 > $O/tests.log 2>&1 || exit $?
