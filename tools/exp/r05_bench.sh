# round 5: the default bench line (C2 legs + the C4r leg), timed by the driver's own clock
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=$(date +%s.%N)
timeout -k 10 1000 python -u bench.py > gpurun_out/r05n_bench.json 2> gpurun_out/r05n_bench.err || { tail -30 gpurun_out/r05n_bench.err; exit 1; }
E=$(date +%s.%N)
echo "bench wall $(echo "$E - $S" | bc) s" >> gpurun_out/r05n_bench.err
