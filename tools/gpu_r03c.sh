set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python tools/ab_gmres.py --rounds 4 --variants "gm_ept=4,gm_ept=5,gm_ept=6,gm_ept=8,gm_ept=0" > $O/ab_gmres.txt 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_gmres.py tests/test_gpu_high_order.py tests/test_partition.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/stats_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 1 --warmup 0 --cg-iters 4 --no-cpu-baseline --no-profile-events --spd-steps 0 --gmres-iters 0 > $O/stats_c3.log 2>&1 || exit $?
