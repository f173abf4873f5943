#!/bin/bash
# SQ counter passes (tools/pmc_sq.sh) of the C2 bench per library build: abtmp/<v>.so for v in VARIANTS,
# into gpurun_out/<TAG>_sq_<v>; the last build is left installed.
set -u
cd "$GRAFT_REPO_ROOT"
LIB=continuum-mechanics-mfem_amd/lib/libcdfem.so
for v in ${VARIANTS:-a b}; do
  cp "abtmp/$v.so" "$LIB" || exit 1
  bash tools/pmc_sq.sh gpurun_out/${TAG:-sq}_sq_$v "$@" || exit $?
done
