set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_high_order.py::test_ho_brick_cg_parity" "tests/test_distributed.py::test_gpu_ho_block_cg_on_slabs" \
  "tests/test_distributed.py::test_gpu_high_order_two_ranks_one_device" > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
for R in 0 9 1 3 11; do
timeout -k 10 200 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --set ho_tile_rot=$R > $O/c3_r${R}_$i.json 2>> $O/bench.err || exit $?
done; done
