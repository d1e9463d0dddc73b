#!/bin/bash
# Round 6: the C4 leg's allocations (PBGPU_DEBUG_STALL=2, PBGPU_DEBUG_BUFFERS=1) to find its
# out-of-memory; the graph kernels' bounds-checking build; the >8192-record read test.
O=gpurun_out/r06d; mkdir -p gpurun_out/r06d
source tools/r06/lib.sh
PBGPU_DEBUG_STALL=2 PBGPU_DEBUG_BUFFERS=1 step c4dbg 400 python3 -u bench.py --only c4 --c4-reads 20000 --device-steps 1 --no-brand
grep -v "^W2026\|^E2026" $O/c4dbg.out | tail -60
step gcheck 900 bash tools/r06/graph_check.sh $O
cat $O/gcheck.out
step bigread 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_mega_reads.py::test_read_past_8192_records_against_restatement
tail -3 $O/bigread.out
cat $O/steps.txt
