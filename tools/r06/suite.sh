#!/bin/bash
# Round 6: the whole -m gpu suite as the driver runs it (one process), log to gpurun_out/r06_suite.log
O=gpurun_out/r06s; mkdir -p gpurun_out/r06s
source tools/r06/lib.sh
step suite 1150 python -u -m pytest tests -m gpu -x -v --timeout 1100 --timeout-method thread
tail -5 $O/suite.out
cat $O/steps.txt
