#!/bin/bash
# Round 6: register LIS for strands of <= 8 hits; bucket partition margin -- parity suites, then
# A/B on C2, C4r and C4.
O=gpurun_out/r06j; mkdir -p gpurun_out/r06j
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fine_details.py tests/test_gpu_golden.py tests/test_gpu_regress.py
tail -3 $O/tests.out
for t in 1 0; do
  PBGPU_LIS_TINY=$t step c2_t$t 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_LIS_TINY=$t step c4r_t$t 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
done
for m in 1.5 1.0 2.0 3.0; do
  PBGPU_GROUP_BUCKET_MARGIN=$m step c4_m$m 400 python3 -u tools/prof_c4.py --reads 50000
done
PBGPU_LIS_TINY=0 step c4_t0 400 python3 -u tools/prof_c4.py --reads 50000
for f in c2_t1 c2_t0 c4r_t1 c4r_t0 c4_m1.5 c4_m1.0 c4_m2.0 c4_m3.0 c4_t0; do echo "== $f"; grep -v "^W2026\|^E2026\|^generate\|^per base" $O/$f.out; done
cat $O/steps.txt
