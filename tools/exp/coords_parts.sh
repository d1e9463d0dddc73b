#!/bin/bash
# k_coords ms per launch for the product library and variants (tools/exp/exp_coords.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base "$@"; do
  lib=pacbio_amd/libpbgpu_$v.so; [ "$v" = base ] && lib=pacbio_amd/libpbgpu.so
  PBGPU_LIB=$lib timeout -k 10 300 python -u tools/exp/exp_coords.py --reps 2 2>&1 | tail -1 || exit 1
done
