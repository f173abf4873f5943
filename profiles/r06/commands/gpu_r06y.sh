set -u
# profiles of the shipped C2 path (pa_uniform: the element matrix on the matrix cores): bench line, rocprof
# stats + per-launch CSV of k_brick_cg, PMC traffic (FETCH / WRITE + calibration), SQ counter passes
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/profile_round.sh r06y c2 || exit $?
D=gpurun_out/prof_r06y_c2
timeout -k 10 120 python3 tools/rocprof_avg.py --trace $D/stats --kernel k_brick_cg --key n64_p2_k7_aff \
    --csv $D/k_brick_cg_launches.csv --json $D/rocprof_kernels.json > $D/rocprof_avg.json || exit $?
bash tools/pmc_sq.sh gpurun_out/r06y_sq_c2 --config c2 > gpurun_out/r06y_sq_c2.log 2>&1 || exit $?
