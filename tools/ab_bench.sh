#!/bin/bash
# Interleaved bench.py A/B of context options on one box: VARIANTS="ho_brick=0 ho_brick=1" ROUNDS=2
#   bash tools/ab_bench.sh OUTDIR [bench args...]  -> OUTDIR/<variant>_<round>.json, a summary line each
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    SETS=""; for kv in ${v//,/ }; do SETS="$SETS --set $kv"; done
    timeout -k 10 600 python bench.py --no-cpu-baseline --spd-steps 0 --per-point-steps 0 --gmres-iters 0 $SETS "$@" \
      > $OUT/${v//[,=]/_}_$r.json 2> $OUT/${v//[,=]/_}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline'].get('other_kernels_avg_us'))" $OUT/${v//[,=]/_}_$r.json "$v" $r
  done
done
