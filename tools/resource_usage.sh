#!/bin/bash
# Per-kernel register / scratch usage of one HIP source (compile remark, gfx950), one line per kernel:
# "name VGPRs AGPRs scratch_bytes_per_lane occupancy".  usage: bash tools/resource_usage.sh csrc/x.hip [regex]
set -eu
cd "$(dirname "$0")/../continuum-mechanics-mfem_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -x hip -c "$1" -o /tmp/ru_$$.o \
    --offload-device-only -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *\(Function Name\|VGPRs\|AGPRs\|ScratchSize \[bytes\/lane\]\|Occupancy \[waves\/SIMD\]\): \([^ ]*\) .*/\1|\2/p' |
  awk -F'|' '$1=="Function Name"{n=$2} $1=="VGPRs"{v=$2} $1=="AGPRs"{a=$2} $1 ~ /^Scratch/{s=$2} $1 ~ /^Occupancy/{print n, v, a, s, $2}' |
  (c++filt 2>/dev/null || cat) | grep -E "${2:-.}" || true
rm -f /tmp/ru_$$.o
