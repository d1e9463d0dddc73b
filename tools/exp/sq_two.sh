#!/bin/bash
# SQ instruction mix of k_coords and k_lis_w (tools/pmc_sq_kernel.sh) for a library variant
set -o pipefail
V=${1:-}
for RE in k_coords k_lis_w; do
  echo "== $RE ${V:-base}"
  bash tools/pmc_sq_kernel.sh $RE $V || exit 1
done
