#!/bin/bash
# Quick GPU check: the named test files, then a short bench.  Usage: bash tools/gpu_quick.sh TAG "tests..." [bench args]
set -o pipefail
TAG=$1; TESTS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
  rc=$?; tail -15 gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$1" != "nobench" ]; then
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err; exit $rc
fi
