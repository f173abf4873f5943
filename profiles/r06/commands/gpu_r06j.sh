set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_brick_cg.py > $O/tests.log 2>&1 || exit $?
for i in 1 2 3; do
for U in 1 0; do
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --set upd_xcd=$U > $O/c2_u${U}_$i.json 2>> $O/bench.err || exit $?
done; done
for U in 1 0; do
timeout -k 10 200 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --set upd_xcd=$U > $O/c3_u${U}.json 2>> $O/bench.err || exit $?
done
