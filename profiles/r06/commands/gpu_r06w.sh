set -u
# pa_uniform apply variants (CDFEM_UM_VARIANT 0 / 1 / 2 builds in abtmp/), each against the Kronecker form in process
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06w; mkdir -p $O
VARIANTS="v0 v1 v2" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --variants pa_uniform=0,pa_uniform=1" 2 > $O/ev.txt 2>&1 || exit $?
cp gpurun_out/ab_v*_*.log $O/ 2>/dev/null
VARIANTS="v0 v1 v2" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --no-events --variants pa_uniform=0,pa_uniform=1" 2 > $O/noev.txt 2>&1 || exit $?
mkdir -p $O/noev; cp gpurun_out/ab_v*_*.log $O/noev/ 2>/dev/null; exit 0
