set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_brick_cg.py "tests/test_distributed.py::test_gpu_mr_fold_grouped_partials" \
  "tests/test_distributed.py::test_gpu_c5_per_rank_slabs" "tests/test_distributed.py::test_gpu_uneven_slabs_fold_toggle" \
  "tests/test_distributed.py::test_gpu_mr_fold_matches_step_kernels" \
  "tests/test_gpu_full_size.py::test_c5_one_gpu_folds_bounded" "tests/test_gpu_full_size.py::test_c5_one_gpu_full_size_oracle_parity" \
  > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 > $O/c5_1gpu.json 2> $O/c5_1gpu.err || exit $?
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --gmres-iters 0 --spd-steps 0 --per-point-steps 0 --set den_group=1 > $O/c5_1gpu_nogroup.json 2>> $O/c5_1gpu.err || exit $?
for F in 1 0; do
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/mrk_f$F -o run --output-format csv -- python3 tools/mr_kernel_list.py --n 256 --per 32 --world 8 --fold $F --iters 30 > $O/mrk_f$F.log 2>&1 || exit $?
python3 tools/mr_kernel_list.py --summary $O/mrk_f$F --world 8 --iters 30 --fold $F >> $O/mr_kernel_list.jsonl || exit $?
done
