#!/bin/bash
# Round 6: the default bench line, then the round's rocprofv3 summary (tools/r06/prof.sh TAG)
TAG=${1:-r06z}
O=gpurun_out/r06b_$TAG; mkdir -p $O
source tools/r06/lib.sh
SECONDS=0
step bench 700 python3 -u bench.py
echo "bench wall $SECONDS s" >> $O/steps.txt
grep '^{"metric"' $O/bench.out | head -c 600; echo
step prof 1000 bash tools/r06/prof.sh $TAG
tail -3 $O/prof.out
cat $O/steps.txt
