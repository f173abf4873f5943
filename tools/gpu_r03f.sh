#!/bin/bash
# round 3f: device-resident time-loop A/B at n = 64, 128, 256 (p = 2), 4 interleaved rounds each
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for N in 64 128 256; do
  timeout -k 10 900 bash tools/ab_time_loop.sh $N 4 > gpurun_out/ab_time_loop_$N.txt 2>&1 || { tail -5 gpurun_out/ab_time_loop_$N.txt; exit 1; }
  echo "n=$N"; grep -o "lib/diffusion_mms .*seconds_per_step [0-9.e-]*\|hostvec .*seconds_per_step [0-9.e-]*" gpurun_out/ab_time_loop_$N.txt | awk '{print $1, $NF}' | tr '\n' ' '; echo
done
