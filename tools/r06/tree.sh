#!/bin/bash
# Round 6: k_lis_tiny's hit pick as a 3-level select tree (variant libpbgpu_tree) against the
# 7-deep select chain (product): LIS stage on C4, C4r, C2; parity
O=gpurun_out/r06tr; mkdir -p gpurun_out/r06tr
source tools/r06/lib.sh
PBGPU_LIB=pacbio_amd/libpbgpu_tree.so step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py
echo "tests tree: $(tail -1 $O/tests.out)"
for rep in 1 2; do
for v in libpbgpu libpbgpu_tree; do
  PBGPU_LIB=pacbio_amd/$v.so step c4_${v}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  PBGPU_LIB=pacbio_amd/$v.so step c4r_${v}_$rep 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  PBGPU_LIB=pacbio_amd/$v.so step c2_${v}_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  for w in c4 c4r c2; do echo "$w $v $rep: $(grep 'stages ms' $O/${w}_${v}_$rep.out | head -1 | cut -c1-200)"; done
done
done
