#!/bin/bash
# Round 6: adaptive record / kmers_info sizing -- parity suites, then the C4 leg (250k reads),
# the graph bounds check, and the C4 leg's kernel trace.
O=gpurun_out/r06e; mkdir -p gpurun_out/r06e
source tools/r06/lib.sh
step tests 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_scale.py tests/test_gpu_fine_details.py
tail -3 $O/tests.out
PBGPU_DEBUG_BUFFERS=1 step c4 500 python3 -u bench.py --only c4 --c4-reads 250000
grep -v "^W2026\|^E2026" $O/c4.out | tail -5 | cut -c1-3000
step gcheck 900 bash tools/r06/graph_check.sh $O
cat $O/graph_check.txt
step c4_trace 500 rocprofv3 --kernel-trace --stats -d $O/c4_trace -o c4 -- python3 -u bench.py --only c4 --c4-reads 100000 --no-brand --device-steps 1
cat $O/steps.txt
