#!/bin/bash
# SQ counters of the C2 bench (kron brick CG) + GMRES path
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/pmc_sq.sh gpurun_out/r04b_sq
python3 tools/pmc_sq_summary.py gpurun_out/r04b_sq > gpurun_out/r04b_sq/summary.json
python3 -c "
import json; d=json.load(open('gpurun_out/r04b_sq/summary.json'))
for k,v in d.items():
    if 'brick' in k or 'update' in k: print(k, json.dumps(v, indent=0)[:3000])
"
