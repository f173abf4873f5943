set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_high_order.py::test_ho_block_z4_parity" "tests/test_gpu_high_order.py::test_ho_brick_cg_parity" \
  > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
for BZ in 4 2; do
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --set ho_block_z=$BZ > $O/c3_bz${BZ}_$i.json 2>> $O/bench.err || exit $?
done; done
