set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_gmres.py > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
for K in 1 2 4 8; do
timeout -k 10 120 python -u bench.py --config c2 --steps 1 --warmup 1 --cg-iters 2 --no-cpu-baseline --spd-steps 0 --per-point-steps 0 --no-profile-events --set gm_poll=$K > $O/c2_k${K}_$i.json 2>> $O/bench.err || exit $?
done; done
for K in 1 4; do
timeout -k 10 200 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --set gm_poll=$K > $O/c4_k${K}.json 2>> $O/bench.err || exit $?
done
