#!/bin/bash
# graph GPU tests, rocprof of the graph kernels (C2 50k), bench's create_mega_reads leg
# (8 runs, stall reports), the C4r host-graph share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mega_reads.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/graph_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/graph_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp/r04_prof_graph.sh $TAG || exit 1
bash tools/exp/cmr_bench_stall.sh $TAG 8 || exit 1
timeout -k 10 400 python3 -u tools/prof_graph_gpu.py --workload C4r --reads 20000 > gpurun_out/c4r_host_share_$TAG.log 2>&1
rc=$?; grep -v "^[EW]20" gpurun_out/c4r_host_share_$TAG.log | tail -3; exit $rc
