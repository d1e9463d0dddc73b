#!/bin/bash
# End-of-round measurement: the default bench line, then the rocprofv3 profile of the
# device leg (tools/prof_r03.sh).  bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 600 gpurun_out/bench_$TAG.json; echo
bash tools/prof_r03.sh $TAG
