#!/bin/bash
# k_group tier-0 ms per library variant (tools/prof_lis.py, non-PROF path): bash tools/exp/ab_group_ms.sh v1 v2 ...
# ("base" = the product libpbgpu.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  lib=pacbio_amd/libpbgpu_$v.so; [ "$v" = base ] && lib=pacbio_amd/libpbgpu.so
  PBGPU_LIB=$lib timeout -k 10 300 python -u tools/prof_lis.py --reads 25000 > gpurun_out/abms_$v.txt 2>&1 || { cat gpurun_out/abms_$v.txt; exit 1; }
  echo "== $v: $(grep k_group gpurun_out/abms_$v.txt)"
done
