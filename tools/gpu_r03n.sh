#!/bin/bash
# round 3n: XCD-contiguous block order of the C3 tile apply (ho_xcd): bitwise test, interleaved A/B,
# and the apply's HBM counters per variant
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03n
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_high_order.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "ho_xcd" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python tools/ab.py --n 128 --p 4 --iters 20 --rounds 4 --variants ho_xcd=0,ho_xcd=1,ho_xcd=0,ho_xcd=1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
grep -E '"ho_xcd|iter_us|"apply"|update' $OUT/ab.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$C -o run --output-format csv -- python3 tools/ab.py --n 128 --p 4 --iters 4 --rounds 0 --no-events --variants ho_xcd=0,ho_xcd=1 > $OUT/pmc_$C.log 2>&1 || exit $?
  f=$(ls $OUT/pmc_$C/*/run_counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$OUT/pmc_$C/run_counter_collection.csv
  cp "$f" $OUT/pmc_$C.csv
done
python tools/pmc_split.py $OUT/pmc_FETCH_SIZE.csv k_apply3d_tile 2 2048
python tools/pmc_split.py $OUT/pmc_WRITE_SIZE.csv k_apply3d_tile 2 1024
