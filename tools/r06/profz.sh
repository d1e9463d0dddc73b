#!/bin/bash
# Round 6: the round's rocprofv3 profile (tools/r06/prof.sh TAG) in a call of its own
TAG=${1:-r06z}
O=gpurun_out/r06p_$TAG; mkdir -p $O
source tools/r06/lib.sh
SECONDS=0
step prof 1150 bash tools/r06/prof.sh $TAG
echo "prof wall $SECONDS s" >> $O/steps.txt
tail -3 $O/prof.out
cat $O/steps.txt
