#!/bin/bash
# Interleaved A/B of two builds of libcdfem.so on one GPU box (for changes that cannot be
# switched at run time, e.g. store flavours or launch bounds).
#   here:    cp <lib A> abtmp/a.so; cp <lib B> abtmp/b.so
#   GPU box: bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --no-events" 3
# Runs A, B, A, B, ... (PAIRS pairs), each under its own time limit, and prints each run's
# iteration / kernel times; the in-tree library is restored to B at the end.  Delete abtmp/
# afterwards (it is sent with every gpurun call).
set -u
cd "$GRAFT_REPO_ROOT"
CMD=${1:?command}
PAIRS=${2:-2}
VARIANTS=${VARIANTS:-"a b"}   # abtmp/<v>.so for each v, interleaved; the last one is left installed
LIB=continuum-mechanics-mfem_amd/lib/libcdfem.so
mkdir -p gpurun_out
for k in $(seq 1 "$PAIRS"); do
  for v in $VARIANTS; do
    cp "abtmp/$v.so" "$LIB" || exit 1
    timeout -k 10 300 $CMD > "gpurun_out/ab_${v}_$k.log" 2>&1 || exit $?
    echo "$v $k: $(grep -hE '"(iter_us|it_us|apply_us|upd_us|spmv_us|orth_us)"' "gpurun_out/ab_${v}_$k.log" | tr -d ' \n')"
  done
done
cp "abtmp/${VARIANTS##* }.so" "$LIB"
