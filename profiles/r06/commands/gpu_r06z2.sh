set -u
# in-process A/B of the one-update (a) and two-update (b) x-fold builds (abtmp/), C2 CG iterations
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06z2; mkdir -p $O
VARIANTS="a b" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --no-events --variants cg_xfold=1" 3 > $O/noev.txt 2>&1 || exit $?
mkdir -p $O/noev; cp gpurun_out/ab_[ab]_*.log $O/noev/
VARIANTS="a b" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --variants cg_xfold=1" 2 > $O/ev.txt 2>&1 || exit $?
cp gpurun_out/ab_[ab]_*.log $O/
