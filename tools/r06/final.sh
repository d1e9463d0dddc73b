#!/bin/bash
# Round 6: parity spot check of the final defaults, then the default bench line (TAG)
TAG=${1:-r06zf}
O=gpurun_out/r06b_$TAG; mkdir -p $O
source tools/r06/lib.sh
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_mega_reads.py -k "bucket or c4 or C4 or overflow or config or long"
tail -1 $O/tests.out
SECONDS=0
step bench 900 python3 -u bench.py
echo "bench wall $SECONDS s" >> $O/steps.txt
grep '^{"metric"' $O/bench.out | head -c 300; echo
cat $O/steps.txt
