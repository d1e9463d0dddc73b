#!/bin/bash
# Round 6: windows a wave and step of the 8- and 16-wave k_group launches (PBGPU_GROUP_U_BIG 2 / 4 / 6)
O=gpurun_out/r06gu; mkdir -p gpurun_out/r06gu
source tools/r06/lib.sh
for rep in 1 2; do
for v in libpbgpu libpbgpu_gu2 libpbgpu_gu6; do
  PBGPU_LIB=pacbio_amd/$v.so step c4_${v}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  echo "c4 $v $rep: $(grep 'stages ms' $O/c4_${v}_$rep.out | head -1 | cut -c1-200)"
done
done
PBGPU_LIB=pacbio_amd/libpbgpu_gu6.so step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py -k "bucket or overflow"
echo "tests gu6: $(tail -1 $O/tests.out)"
