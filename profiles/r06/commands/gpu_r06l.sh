# round-6 records of the shipped kernels: bench lines + rocprof per-launch CSVs (c2, c3), SQ passes (c2)
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/profile_r06.sh r06l c2 || exit $?
bash tools/profile_r06.sh r06l c3 || exit $?
bash tools/pmc_sq.sh gpurun_out/r06l_sq_c2 > gpurun_out/r06l_sq_c2.log 2>&1 || exit $?
