#!/bin/bash
# Round 6: the default bench line alone (as the driver runs it), wall time recorded
TAG=${1:-r06z}
O=gpurun_out/r06b_$TAG; mkdir -p $O
source tools/r06/lib.sh
SECONDS=0
step bench 1100 python3 -u bench.py
echo "bench wall $SECONDS s" >> $O/steps.txt
grep '^{"metric"' $O/bench.out | head -c 400; echo
cat $O/steps.txt
