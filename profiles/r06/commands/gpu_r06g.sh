set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06g; mkdir -p $O
for i in 1 2; do
for ST in 0 $((8 | 2<<4)) $((8 | 4<<4)) $((10 | 2<<4)) $((10 | 4<<4)) $((0 | 2<<4)) $((0 | 4<<4)) $((7 | 3<<4)); do
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --set brick_stagger=$ST > $O/c2_st${ST}_$i.json 2>> $O/bench.err || exit $?
done; done
