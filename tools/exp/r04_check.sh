#!/bin/bash
# Round-4 check: parity subset (everything but C4/C5 scale and the multi-index suites), then
# the graph kernel profile and the k_coords A/B of the named variants
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-c}; shift
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py tests/test_gpu_fine_details.py \
  tests/test_gpu_golden.py tests/test_gpu_mega_reads.py tests/test_gpu_regress.py > gpurun_out/check_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/check_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/r04_prof_graph.sh $TAG || exit 1
bash tools/exp/coords_parts.sh "$@"
