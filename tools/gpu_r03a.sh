set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r03a
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/r03a/bench_c2.json 2> gpurun_out/r03a/bench_c2.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03a/stats -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-events --spd-steps 0 > gpurun_out/r03a/stats.log 2>&1 || exit $?
