# round 5: the bench line (defaults: N=1, the C2 workload, every leg) and a rocprofv3 kernel-stats pass of it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err || { tail -30 gpurun_out/r05_bench.err; exit 1; }
tail -1 gpurun_out/r05_bench.json | cut -c1-400
