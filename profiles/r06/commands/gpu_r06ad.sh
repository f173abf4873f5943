set -u
# brick_tile (3D-tile brick order of the p <= 2 apply): bitwise tests, then bench A/B at C5 and C2 and C5's traffic with tiles
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06ad; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_brick_cg.py::test_brick_tile_order_bitwise" > $O/tests.log 2>&1 || exit $?
VARIANTS="brick_tile=0 brick_tile=1" ROUNDS=2 bash tools/ab_bench.sh $O/c5 --config c5 --steps 2 --warmup 1 > $O/c5.log 2>&1 || exit $?
VARIANTS="brick_tile=0 brick_tile=1" ROUNDS=2 bash tools/ab_bench.sh $O/c2 > $O/c2.log 2>&1 || exit $?
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -d $O/pmc_fetch_t1 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --cg-iters 10 --gmres-iters 0 --spd-steps 0 --no-cpu-baseline --no-profile-events --no-kron-form --per-point-steps 0 --set brick_tile=1 > $O/pmc_fetch_t1.log 2>&1 || exit $?
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -d $O/pmc_write_t1 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --cg-iters 10 --gmres-iters 0 --spd-steps 0 --no-cpu-baseline --no-profile-events --no-kron-form --per-point-steps 0 --set brick_tile=1 > $O/pmc_write_t1.log 2>&1 || exit $?
