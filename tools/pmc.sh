#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only — MI355X_MICROARCH.md §rocprofv3 PMC):
# HBM bytes of the hot kernels (FETCH_SIZE / WRITE_SIZE, corrected per the guide's gfx950 notes)
# plus wave-cycle breakdown.  Writes gpurun_out/pmc_<path>_<pass>/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PATHS=${1:-brick}
ARGS="--steps 1 --warmup 0 --cg-iters 20 --no-profile-events --no-cpu-baseline"
for P in $PATHS; do
  i=0
  for G in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace -T -d gpurun_out/pmc_${P}_$i -o run --output-format csv -- python3 bench.py $ARGS --path $P > gpurun_out/pmc_${P}_$i.log 2>&1 || exit $?
  done
done
exit 0
