#!/bin/bash
# Round 6: the register LIS for strands of <= 12 hits (PBGPU_LIS_LANE_MAX=12) against <= 8
O=gpurun_out/r06ln; mkdir -p gpurun_out/r06ln
source tools/r06/lib.sh
PBGPU_LIB=pacbio_amd/libpbgpu_ln12.so step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_parity.py
echo "tests ln12: $(tail -1 $O/tests.out)"
for rep in 1 2; do
for v in libpbgpu libpbgpu_ln12; do
  PBGPU_LIB=pacbio_amd/$v.so step c4_${v}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  PBGPU_LIB=pacbio_amd/$v.so step c2_${v}_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  for w in c4 c2; do echo "$w $v $rep: $(grep 'stages ms' $O/${w}_${v}_$rep.out | head -1 | cut -c1-200)"; done
done
done
