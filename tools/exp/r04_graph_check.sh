#!/bin/bash
# create_mega_reads GPU tests, then the C2 create_mega_reads timing (tools/bench_cmr.py-like: 3 cold runs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mega_reads.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/graph_tests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/graph_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --device-steps 1 --parts 0 --cmr-steps 3 --no-cpu-baseline --no-brand --skip-default-leg > gpurun_out/graph_bench_$TAG.json 2> gpurun_out/graph_bench_$TAG.err
rc=$?
python3 -c "
import json; d=json.load(open('gpurun_out/graph_bench_$TAG.json'))
print('cmr', d['value_create_mega_reads']/1e9, d['create_mega_reads_walls_s'], d['create_mega_reads_stage_s'])" || tail -5 gpurun_out/graph_bench_$TAG.err
exit $rc
