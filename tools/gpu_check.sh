#!/bin/bash
# Quick GPU check of a kernel change: parity subset, then k_group tier-0 ms of libraries.
#   bash tools/gpu_check.sh "tests/test_gpu_parity.py tests/test_gpu_edge.py" base r03h
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TESTS=$1; shift
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/check_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/check_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ $# -gt 0 ]; then bash tools/exp/ab_group_ms.sh "$@"; fi
