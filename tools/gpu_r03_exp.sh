#!/bin/bash
# bench (no CPU leg) + create_mega_reads bench + k_group variants' tier-0 ms.  bash tools/gpu_r03_exp.sh TAG [variants...]
set -o pipefail
TAG=${1:-r03}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 400 gpurun_out/bench_$TAG.json; echo
timeout -k 10 300 python -u tools/bench_cmr.py > gpurun_out/cmr_$TAG.json 2>&1 || { tail -20 gpurun_out/cmr_$TAG.json; exit 1; }
cat gpurun_out/cmr_$TAG.json
[ $# -gt 0 ] && bash tools/exp/ab_group_ms.sh "$@"
