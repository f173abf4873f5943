set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_brick_cg.py::test_brick_mfma_x_stage_parity" > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
for MX in 1 0; do
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --set brick_mfma=$MX > $O/c2_mx${MX}_$i.json 2>> $O/bench.err || exit $?
done; done
bash tools/pmc_sq.sh $O/sq_mx1 --set brick_mfma=1 > $O/sq_mx1.log 2>&1 || exit $?
bash tools/pmc_sq.sh $O/sq_mx0 --set brick_mfma=0 > $O/sq_mx0.log 2>&1 || exit $?
