set -u
# C5 (256^3 p = 2, one GPU) profile on the uniform element matrix: bench, rocprof stats + per-launch CSV, PMC traffic
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/profile_round.sh r06ac c5 || exit $?
D=gpurun_out/prof_r06ac_c5
timeout -k 10 120 python3 tools/rocprof_avg.py --trace $D/stats --kernel k_brick_cg --key n256_p2_k7_aff \
    --csv $D/k_brick_cg_launches.csv --json $D/rocprof_kernels.json > $D/rocprof_avg.json || exit $?
