set -u
# first-round stagger re-tuned for the MFMA apply: off, 2, 4 (auto), 6 sleeps of 2,048 cycles (shift 8 = log2 256 CUs)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06af; mkdir -p $O
VARIANTS="brick_stagger=0 brick_stagger=40 brick_stagger=72 brick_stagger=104" ROUNDS=2 bash tools/ab_bench.sh $O/ab > $O/ab.log 2>&1 || exit $?
