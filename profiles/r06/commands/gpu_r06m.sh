set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gm -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 0 --cg-iters 2 --spd-steps 0 --per-point-steps 0 --no-cpu-baseline --no-profile-events --gmres-iters 60 > $O/gm.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gm4 -o run --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events > $O/gm4.log 2>&1 || exit $?
