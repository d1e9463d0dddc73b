#!/bin/bash
# rocprofv3 kernel stats + HBM PMC passes of bench.py (full C2 workload).
# Usage (via gpurun): bash tools/prof_round.sh TAG
set -o pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/prof_$TAG
mkdir -p $D
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- $B > $D/bench.json 2> $D/kt.err || { tail -20 $D/kt.err; exit 1; }
cat $D/bench.json
P="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/p_fetch -o run -- $P > $D/p_fetch.log 2>&1 || { tail -20 $D/p_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/p_write -o run -- $P > $D/p_write.log 2>&1 || { tail -20 $D/p_write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $D/p_tcc -o run -- $P > $D/p_tcc.log 2>&1 || { tail -20 $D/p_tcc.log; exit 1; }
ls -R $D | head -40
