#!/bin/bash
# C3 (128^3 p=4): MFMA stages on the affine-factor tile apply, in-process A/B
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04i}; mkdir -p $O
timeout -k 10 600 python -u tools/ab.py --n 128 --p 4 --iters 10 --rounds 3 --variants "ho_mfma=0,ho_mfma=1,ho_mfma=8,ho_mfma=9" > $O/ab_c3_mfma.json 2> $O/ab_c3_mfma.err || { echo "ab rc=$?"; tail $O/ab_c3_mfma.err; exit 1; }
cat $O/ab_c3_mfma.json
