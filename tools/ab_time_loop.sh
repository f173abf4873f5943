#!/bin/bash
# diffusion_mms time loop, device-resident Vectors (lib/diffusion_mms) against the same driver built
# on the round-2 host-vector shim (ab_bin/diffusion_mms_hostvec, built from git by the caller),
# interleaved, 10 backward-Euler steps on an n x n quad mesh at p = 2.  Prints seconds_per_step.
# usage: bash tools/ab_time_loop.sh [n] [rounds]
set -u
cd "$GRAFT_REPO_ROOT"
N=${1:-512}
R=${2:-3}
OPTS=gpurun_out/ab_tl_petsc.opts
mkdir -p gpurun_out
printf -- "-ksp_type gmres\n-ksp_rtol 1.0e-10\n-ksp_atol 1.0e-12\n-ksp_max_it 5000\n-pc_type jacobi\n" > $OPTS
for r in $(seq 1 $R); do
  for exe in continuum-mechanics-mfem_amd/lib/diffusion_mms ab_bin/diffusion_mms_hostvec; do
    out=$(CDFEM_SHIM_STATS=1 timeout -k 10 300 $exe -n $N -p 2 -dt 0.005 -T 0.05 -opts $OPTS 2>&1) || { echo "$exe failed: $out"; exit 1; }
    echo "round $r $exe $(echo "$out" | grep -E 'seconds_per_step|final_l2|gmres_iterations|shim_transfers' | tr '\n' ' ')"
  done
done
