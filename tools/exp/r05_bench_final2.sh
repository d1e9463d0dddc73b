# round 5 (after the edge-scan prefilter): the bench line (defaults: N=1, the C2 workload, every leg)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r05_bench3.json 2> gpurun_out/r05_bench3.err || { tail -30 gpurun_out/r05_bench3.err; exit 1; }
tail -1 gpurun_out/r05_bench3.json | cut -c1-300
