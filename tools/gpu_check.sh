set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
nproc > gpurun_out/nproc.txt
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench1.log
exit $rc
