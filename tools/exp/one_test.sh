#!/bin/bash
# one GPU test (node id as the argument), verbose
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/one_test.log 2>&1
rc=$?; tail -15 gpurun_out/one_test.log; exit $rc
