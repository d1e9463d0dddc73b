#!/bin/bash
# Round 6: last check of the in-tree library: smoke() and the parity files
O=gpurun_out/r06last; mkdir -p gpurun_out/r06last
source tools/r06/lib.sh
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.out
step tests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_mega_reads.py
tail -1 $O/tests.out
