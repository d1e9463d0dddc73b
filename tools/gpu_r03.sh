#!/bin/bash
# Round-3 GPU session: the -m gpu suite (optionally a -k filter), then (optional) smoke + bench.
#   tools/gpu_r03.sh TAG [KFILTER] [bench]
set -o pipefail
TAG=${1:-r03}
K=${2:-"not c5"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$K" \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
if [ "$3" = "bench" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
  cat gpurun_out/smoke_$TAG.log
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi
