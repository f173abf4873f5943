#!/bin/bash
# C2 A/B after the predicated update: x-fold and three waves per SIMD re-measured; C3 profile.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r04r}; mkdir -p $O
timeout -k 10 300 python -u tools/ab_opts.py --variant "cg_xfold=0" --variant "cg_xfold=1" --variant "brick_cg_waves=3" --rounds 5 --iters 100 > $O/ab_c2_xfold_waves.json 2> $O/ab_c2.err || { echo "ab rc=$?"; tail $O/ab_c2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_c2_xfold_waves.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b,2) if isinstance(b,float) else b) for a,b in v.items() if a!='it_us_all'})
"
bash tools/gpu_r04_prof.sh c3
