set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_high_order.py tests/test_gpu_rccl.py tests/test_gpu_fa.py tests/test_cpp_driver.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python tools/ab.py --n 128 --p 4 --rounds 4 --iters 20 --variants "e2l_flat=0,e2l_flat=1" > $O/ab_flat.txt 2>&1 || exit $?
timeout -k 10 400 python tools/ab_c4.py --rounds 4 --variants "l1:natural:spmv_lpr=1,l2:natural:spmv_lpr=2,l4:natural:spmv_lpr=4,l1b:natural:spmv_lpr=1,l4b:natural:spmv_lpr=4" > $O/ab_c4.txt 2>&1 || exit $?
