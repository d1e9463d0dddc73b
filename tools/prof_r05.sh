#!/bin/bash
# Round-5 profile of the bench (as tools/prof_r03.sh, the C4r leg off): rocprofv3 kernel trace + stats, then separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) over the five timed kernels of the production
# device leg (--skip-default-leg: every large-grid launch is that leg's), and the
# FETCH_SIZE calibration on the gather microbenchmarks; summary by
# tools/rocprof_summary.py into gpurun_out/prof_TAG/TAG_{rocprof_summary.json,kernel_stats.txt}.
# Usage (via gpurun): bash tools/prof_r05.sh TAG
set -o pipefail
TAG=${1:-r05z}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --skip-default-leg --cmr-steps 0 --c4r-reads 0 --parts 0 > $D/bench.json 2> $D/kt.err || { tail -20 $D/kt.err; exit 1; }
echo "kernel trace done"
B="python3 bench.py --steps 1 --warmup 0 --device-steps 1 --no-cpu-baseline --no-brand --skip-default-leg --cmr-steps 0 --c4r-reads 0 --parts 0"
RE="k_seed|k_group|k_lis_w|k_coords|k_rec_sort|k_gather"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RE" --output-format csv -d $D/p_$C -o run -- $B > $D/p_$C.log 2>&1 || { tail -20 $D/p_$C.log; exit 1; }
  echo "pmc $C done"
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gather" --output-format csv -d $D/p_cal -o run -- python3 tools/calib_gather.py > $D/p_cal.log 2>&1 || { tail -20 $D/p_cal.log; exit 1; }
python3 tools/rocprof_summary.py $D $D $TAG
