#!/bin/bash
# Per-kernel ms (tools/exp/kernel_ms.py, 25k C2 reads) of the product library under
# environment settings, interleaved twice: bash tools/exp/ab_env.sh "" "PBGPU_OCC_SR=1" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python -u tools/exp/kernel_ms.py --reads 25000 > gpurun_out/abenv.txt 2>&1 || { cat gpurun_out/abenv.txt; exit 1; }
    echo "[$e] $(tail -1 gpurun_out/abenv.txt)"
  done
done
