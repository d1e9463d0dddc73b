#!/bin/bash
# Round-6 profile of the bench (as tools/prof_r05.sh; the C4r / C3 / C4 legs off): rocprofv3 kernel
# trace + stats of the C2 device leg, separate FETCH_SIZE / WRITE_SIZE passes over its five timed
# kernels, the gather calibrations; summary by tools/rocprof_summary.py into
# gpurun_out/prof_TAG/TAG_{rocprof_summary.json,kernel_stats.txt}.  Then the C4 leg: kernel
# trace (csv) and FETCH / WRITE passes of its kernels -> gpurun_out/prof_TAG/c4_*.
# Usage (via gpurun): bash tools/r06/prof.sh TAG
set -o pipefail
TAG=${1:-r06z}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/prof_$TAG
mkdir -p $D
OFF="--c4r-reads 0 --c3-reads 0 --c4-reads 0 --parts 0 --cmr-steps 0"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --skip-default-leg $OFF > $D/bench.json 2> $D/kt.err || { tail -20 $D/kt.err; exit 1; }
echo "kernel trace done"
B="python3 bench.py --steps 1 --warmup 0 --device-steps 1 --no-cpu-baseline --no-brand --skip-default-leg $OFF"
RE="k_seed|k_group|k_lis_w|k_coords|k_rec_sort|k_gather"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RE" --output-format csv -d $D/p_$C -o run -- $B > $D/p_$C.log 2>&1 || { tail -20 $D/p_$C.log; exit 1; }
  echo "pmc $C done"
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gather" --output-format csv -d $D/p_cal -o run -- python3 tools/calib_gather.py > $D/p_cal.log 2>&1 || { tail -20 $D/p_cal.log; exit 1; }
python3 tools/rocprof_summary.py $D $D $TAG || exit 1
# the C4 leg (100k reads, one timed pass)
C4="python3 -u bench.py --only c4 --c4-reads 100000 --no-brand --device-steps 1"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c4_kt -o run -- $C4 > $D/c4.json 2> $D/c4_kt.err || { tail -20 $D/c4_kt.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "k_seed|k_group|k_lis|k_coords|k_rec" --output-format csv -d $D/c4_$C -o run -- $C4 > $D/c4_$C.log 2>&1 || { tail -20 $D/c4_$C.log; exit 1; }
  echo "c4 pmc $C done"
done
echo ok
