#!/bin/bash
# Round-4 profiles: bench + rocprofv3 kernel stats + PMC traffic passes (tools/profile_round.sh) and
# SQ counter passes (tools/pmc_sq.sh) for one config; optional N=8 --comm host rehearsal (8 ranks
# sharing the one GPU over the host communicator; C5's 256^3 split into eight slabs).
# usage: bash tools/gpu_r04_prof.sh CFG [rehearsal]
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
CFG=$1
timeout -k 10 1000 bash tools/profile_round.sh r04 $CFG || { echo "profile_round rc=$?"; exit 1; }
echo "profile_round $CFG done"
case $CFG in
  c2) SQA="";;
  c3) SQA="--config c3 --cg-iters 4";;
esac
timeout -k 10 900 bash tools/pmc_sq.sh gpurun_out/r04_sq_$CFG $SQA || { echo "pmc_sq rc=$?"; exit 1; }
echo "pmc_sq $CFG done"
if [ "${2:-}" = rehearsal ]; then
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 8 --comm host --config c5 --steps 3 --warmup 1 \
      > gpurun_out/r04_rehearsal_n8_c5.json 2> gpurun_out/r04_rehearsal_n8_c5.err || { echo "rehearsal rc=$?"; tail gpurun_out/r04_rehearsal_n8_c5.err; exit 1; }
  cut -c1-300 gpurun_out/r04_rehearsal_n8_c5.json
fi
