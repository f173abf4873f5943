set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_gmres.py > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
for V in "1 1" "8 1" "1 0" "8 0" "4 0"; do
set -- $V
timeout -k 10 120 python -u bench.py --config c2 --steps 1 --warmup 1 --cg-iters 2 --no-cpu-baseline --spd-steps 0 --per-point-steps 0 --no-profile-events --set gm_poll=$1 --set gm_pfence=$2 > $O/c2_k$1_f$2_$i.json 2>> $O/bench.err || exit $?
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gm -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 0 --cg-iters 2 --spd-steps 0 --per-point-steps 0 --no-cpu-baseline --no-profile-events --gmres-iters 60 --set gm_poll=8 --set gm_pfence=0 > $O/gm.log 2>&1 || exit $?
