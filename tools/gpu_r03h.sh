#!/bin/bash
# round 3h: in-launch grid sums (grid_fin): GPU suite, then interleaved A/B on the C2 CG and GMRES legs
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03h
mkdir -p $OUT
T=800 bash tools/gpu_suite.sh; rc=$?
cp gpurun_out/suite.log $OUT/suite.log
tail -3 $OUT/suite.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab.py --no-events --rounds 6 --variants grid_fin=0,grid_fin=1 > $OUT/ab_cg.txt 2>&1 || exit $?
tail -4 $OUT/ab_cg.txt
timeout -k 10 300 python tools/ab_gmres.py --no-prof --rounds 6 --variants grid_fin=0,grid_fin=1 > $OUT/ab_gmres.txt 2>&1 || exit $?
tail -4 $OUT/ab_gmres.txt
timeout -k 10 300 python tools/ab_gmres.py --no-prof --rounds 6 --variants gm_faces=0,gm_faces=1 > $OUT/ab_gmres_faces.txt 2>&1 || exit $?
tail -4 $OUT/ab_gmres_faces.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile-events --spd-steps 0 --cg-iters 6 --gmres-iters 60 > $OUT/c2.log 2>&1 || exit $?
cp $OUT/c2/run_kernel_trace.csv $OUT/c2_kernel_trace.csv 2>/dev/null || cp $OUT/c2/*/run_kernel_trace.csv $OUT/c2_kernel_trace.csv
