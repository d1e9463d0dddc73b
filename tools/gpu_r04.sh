#!/bin/bash
# Round-4 GPU session: the whole -m gpu suite, smoke, the bench, then the rocprofv3
# kernel stats and PMC passes of the bench's device leg (tools/prof_r03.sh, tag r04).
set -o pipefail
TAG=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/suite_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/suite_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/suite_$TAG.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 700 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['value_device'], d['value_create_mega_reads'], d['roofline']['frac'])"
