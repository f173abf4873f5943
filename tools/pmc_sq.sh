#!/bin/bash
# SQ counter passes for one bench configuration (kernel-trace only, <= 8 SQ counters per pass,
# MI355X_MICROARCH.md rocprofv3 section): wave-cycle breakdown, instruction mix, LDS.
# usage: bash tools/pmc_sq.sh OUTDIR [bench args...]   -> OUTDIR/sq_<i>/run_counter_collection.csv
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --cg-iters 20 --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --no-profile-events --no-cpu-baseline --no-kron-form $*"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD" \
         "SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INST_LEVEL_VMEM SQ_INSTS_FLAT" \
         "SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"; do
  i=$((i+1))
  if [ -s $OUT/counters_list.txt ]; then  # keep only the counters this box lists
    H=""; for c in $G; do grep -qw "$c" $OUT/counters_list.txt && H="$H $c"; done; G=$H
  fi
  echo "pass $i: $G" >> $OUT/passes.txt
  [ -z "$G" ] && continue
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $G --kernel-trace -T -d $OUT/sq_$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/sq_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/sq_$i.log; }
done
exit 0
