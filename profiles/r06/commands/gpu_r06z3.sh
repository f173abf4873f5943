set -u
# in-process A/B: one-update x-fold (a), two-update (b), two-update with the two-half gather on its MFMA apply (c)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06z3; mkdir -p $O
VARIANTS="a b c" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --no-events --variants cg_xfold=1" 3 > $O/noev.txt 2>&1 || exit $?
mkdir -p $O/noev; cp gpurun_out/ab_[abc]_*.log $O/noev/
VARIANTS="a b c" bash tools/ab_libs.sh "python tools/ab.py --rounds 4 --iters 100 --variants cg_xfold=1" 2 > $O/ev.txt 2>&1 || exit $?
cp gpurun_out/ab_[abc]_*.log $O/
