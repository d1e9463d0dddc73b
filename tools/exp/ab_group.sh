#!/bin/bash
# A/B of k_group variants: single-stream phase profile (prof lib) + parity subset
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  PBGPU_GROUP_STAGE=$v timeout -k 10 300 python -u tools/prof_lis.py --reads 25000 > gpurun_out/ab_group_$v.txt 2>&1 || { cat gpurun_out/ab_group_$v.txt; exit 1; }
  echo "== PBGPU_GROUP_STAGE=$v"; grep -A6 "2048-slot" gpurun_out/ab_group_$v.txt
done
