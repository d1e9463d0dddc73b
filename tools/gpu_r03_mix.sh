#!/bin/bash
# Round 3: a -k filtered set of GPU tests, then C5 (tools/gpu_c5.sh).  tools/gpu_r03_mix.sh TAG "KFILTER" [SHARDS]
set -o pipefail
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
bash tools/gpu_c5.sh $TAG ${3:-16} 1000
