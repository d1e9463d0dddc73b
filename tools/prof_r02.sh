#!/bin/bash
# Round-2 profile: rocprofv3 kernel trace + stats of the bench command, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) of a short bench and
# of the gather calibration microbenchmarks.  Usage (via gpurun): bash tools/prof_r02.sh TAG
set -o pipefail
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/kt.err || { tail -20 $D/kt.err; exit 1; }
cat $D/bench.json
B="python3 bench.py --steps 1 --warmup 0 --device-steps 1 --no-cpu-baseline --no-brand"
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $C | tr ' ' '_')
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_group|k_gather|k_coords" --output-format csv -d $D/p_$n -o run -- $B > $D/p_$n.log 2>&1 || { tail -20 $D/p_$n.log; exit 1; }
  echo "pmc $C done"
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gather" --output-format csv -d $D/p_cal -o run -- python3 tools/calib_gather.py > $D/p_cal.log 2>&1 || { tail -20 $D/p_cal.log; exit 1; }
python3 tools/rocprof_summary.py $D $D
