#!/bin/bash
# Full GPU suite + smoke, as the driver runs them at round end (timed).  bash tools/gpu_suite.sh TAG
set -o pipefail
TAG=${1:-suite}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
t0=$(date +%s)
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > gpurun_out/suite_$TAG.log 2>&1
rc=$?; t1=$(date +%s); echo "suite rc=$rc in $((t1-t0)) s"; tail -25 gpurun_out/suite_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3
