set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gm30 -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 0 --cg-iters 2 --spd-steps 0 --per-point-steps 0 --no-cpu-baseline --no-profile-events --gmres-iters 60 --set gm_poll=30 > $O/gm30.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gm1 -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 0 --cg-iters 2 --spd-steps 0 --per-point-steps 0 --no-cpu-baseline --no-profile-events --gmres-iters 60 --set gm_poll=1 > $O/gm1.log 2>&1 || exit $?
