set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_gmres.py "tests/test_gpu_full_size.py::test_c4_full_size_parity" tests/test_distributed.py \
  tests/test_reference_inputs.py tests/test_cpp_driver.py tests/test_gpu_fa.py > $O/tests.log 2>&1 || exit $?
