set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/stats_c2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-events --spd-steps 0 > $O/stats_c2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/stats_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-profile-events --spd-steps 0 --gmres-iters 0 > $O/stats_c3.log 2>&1 || exit $?
