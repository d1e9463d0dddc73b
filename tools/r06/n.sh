#!/bin/bash
# Round 6: bucketing from P >= 2 with 2048-slot items -- parity suites, timings, C4 kernel trace.
O=gpurun_out/r06n; mkdir -p gpurun_out/r06n
source tools/r06/lib.sh
step tests 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_fine_details.py tests/test_gpu_mega_reads.py
tail -2 $O/tests.out
step c2 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
step c4r 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
step c4 400 python3 -u tools/prof_c4.py --reads 50000
for f in c2 c4r c4; do echo "== $f: $(grep -v "^W2026\|^E2026\|^generate\|^per base" $O/$f.out | tr '\n' ' ')"; done
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c4 -- python3 -u tools/prof_c4.py --reads 50000
cat $O/steps.txt
