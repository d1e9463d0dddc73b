#!/bin/bash
O=gpurun_out/r06edge; mkdir -p gpurun_out/r06edge
source tools/r06/lib.sh
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py
grep -E "PASSED|FAILED|passed|failed" $O/tests.out | tail -12
