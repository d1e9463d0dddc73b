#!/bin/bash
# phase profile (tools/prof_lis.py) under several library variants: bash tools/exp/ab_libs.sh prof prof_x ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  PBGPU_LIB=pacbio_amd/libpbgpu_$v.so timeout -k 10 300 python -u tools/prof_lis.py --reads 25000 > gpurun_out/ab_$v.txt 2>&1 || { cat gpurun_out/ab_$v.txt; exit 1; }
  echo "== $v"; grep -A5 "2048-slot" gpurun_out/ab_$v.txt; grep "^k_lis:" gpurun_out/ab_$v.txt
done
