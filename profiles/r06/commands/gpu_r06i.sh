set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_brick_cg.py tests/test_gpu_full_size.py::test_c2_headline_full_size_parity > $O/tests.log 2>&1 || exit $?
for i in 1 2 3; do
for ST in -1 0; do
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --spd-steps 0 --per-point-steps 0 --set brick_stagger=$ST > $O/c2_st${ST}_$i.json 2>> $O/bench.err || exit $?
done; done
