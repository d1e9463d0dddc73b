# round 5: the bench line (defaults: N=1, the C2 workload, every leg), then a kernel trace of the C4r
# resident call with its graph
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err || { tail -30 gpurun_out/r05_bench.err; exit 1; }
tail -1 gpurun_out/r05_bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05zk_prof -o c4r -- python3 tools/prof_graph_gpu.py --workload C4r --reads 20000 > gpurun_out/r05zk_graph.txt 2>&1 || exit 1
