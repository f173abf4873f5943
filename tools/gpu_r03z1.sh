#!/bin/bash
# round 3 final profiles, part 1: C2 (bench + kernel stats + PMC passes) and two more C2 bench lines
# (cpu_baseline reproducibility across runs)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/profile_round.sh r03z c2 || exit $?
for k in 2 3; do
  timeout -k 10 600 python bench.py > gpurun_out/prof_r03z_c2/bench_run$k.json 2> gpurun_out/prof_r03z_c2/bench_run$k.err || exit $?
done
cat gpurun_out/prof_r03z_c2/bench.json | head -c 600; echo
