set -u
# MX 2 apply with node 26 through lane shuffles (13.3 KB of LDS, 3 waves per SIMD: b) against the shipped one-trip form (a)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06ae; mkdir -p $O
VARIANTS="a b" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --no-events --variants pa_uniform=1" 3 > $O/noev.txt 2>&1 || exit $?
mkdir -p $O/noev; cp gpurun_out/ab_[ab]_*.log $O/noev/
VARIANTS="a b" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --variants pa_uniform=1" 2 > $O/ev.txt 2>&1 || exit $?
cp gpurun_out/ab_[ab]_*.log $O/
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_uniform.py tests/test_gpu_full_size.py > $O/tests.log 2>&1 || exit $?
