#!/bin/bash
O=gpurun_out/r06late2; mkdir -p gpurun_out/r06late2
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_mega_reads.py tests/test_gpu_edge.py tests/test_gpu_streams.py
tail -1 $O/tests.out
