#!/bin/bash
# Per-kernel ms per library variant (tools/exp/kernel_ms.py): bash tools/exp/ab_kernels.sh v1 v2 ...
# ("base" = the product libpbgpu.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  lib=pacbio_amd/libpbgpu_$v.so; [ "$v" = base ] && lib=pacbio_amd/libpbgpu.so
  PBGPU_LIB=$lib timeout -k 10 300 python -u tools/exp/kernel_ms.py > gpurun_out/abk_$v.txt 2>&1 || { cat gpurun_out/abk_$v.txt; exit 1; }
  echo "== $v: $(tail -1 gpurun_out/abk_$v.txt)"
done
