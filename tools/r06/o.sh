#!/bin/bash
# Round 6: LIS strand ranges and k_coords chain info from the permutation passes -- parity, A/B.
O=gpurun_out/r06o; mkdir -p gpurun_out/r06o
source tools/r06/lib.sh
step tests 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fine_details.py tests/test_gpu_golden.py tests/test_gpu_regress.py tests/test_gpu_scale.py
tail -2 $O/tests.out
step c2 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
step c4r 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
step c4 400 python3 -u tools/prof_c4.py --reads 50000
for f in c2 c4r c4; do echo "== $f: $(grep -v "^W2026\|^E2026\|^generate\|^per base" $O/$f.out | tr '\n' ' ')"; done
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c4 -- python3 -u tools/prof_c4.py --reads 50000
cat $O/steps.txt
