set -u
# GMRES leg timed without the breakdown events (bench.py), C2 default bench twice + a kernel trace
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06u; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 bench.py > $O/c2_$i.json 2> $O/c2_$i.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gm -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 0 --cg-iters 2 --spd-steps 0 --per-point-steps 0 --no-cpu-baseline --no-profile-events --gmres-iters 60 > $O/gm.log 2>&1 || exit $?
