#!/bin/bash
# C5 on one GPU (tests/test_gpu_c5.py), progress and timings under gpurun_out/c5_TAG/.
#   tools/gpu_c5.sh TAG [SHARDS] [READS]
set -o pipefail
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c5_$TAG
export PBGPU_TEST_OUT=gpurun_out/c5_$TAG PBGPU_C5_SHARDS=${2:-16} PBGPU_C5_READS=${3:-1000}
timeout -k 10 1100 python -u -m pytest tests/test_gpu_c5.py -m gpu -x -v -s --timeout 1080 --timeout-method thread \
  > gpurun_out/c5_$TAG/pytest.log 2>&1 || { tail -60 gpurun_out/c5_$TAG/pytest.log; exit 1; }
tail -8 gpurun_out/c5_$TAG/pytest.log
