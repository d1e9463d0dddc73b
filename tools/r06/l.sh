#!/bin/bash
# Round 6: register LIS up to 12 / 15 hits (variants) against 8 (product); the bucket threshold
# on C4; parity with the 15 variant.
O=gpurun_out/r06l; mkdir -p gpurun_out/r06l
source tools/r06/lib.sh
PBGPU_GROUP_BUCKET_LOG2=11 step tests_lg11 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py
tail -2 $O/tests_lg11.out
PBGPU_LIB=pacbio_amd/libpbgpu_lane15.so step tests15 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_regress.py
tail -2 $O/tests15.out
for v in libpbgpu libpbgpu_lane12 libpbgpu_lane15; do
  PBGPU_LIB=pacbio_amd/$v.so step c2_$v 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_LIB=pacbio_amd/$v.so step c4r_$v 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  PBGPU_LIB=pacbio_amd/$v.so step c4_$v 400 python3 -u tools/prof_c4.py --reads 50000
done
PBGPU_GROUP_BUCKET_MINP=2 step c4_mp2 400 python3 -u tools/prof_c4.py --reads 50000
for lg in 11 12; do
  PBGPU_GROUP_BUCKET_LOG2=$lg step c4_lg$lg 400 python3 -u tools/prof_c4.py --reads 50000
  PBGPU_GROUP_BUCKET_LOG2=$lg step c4r_lg$lg 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  PBGPU_GROUP_BUCKET_LOG2=$lg step c2_lg$lg 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
done
for f in c2_libpbgpu c2_libpbgpu_lane12 c2_libpbgpu_lane15 c2_lg11 c2_lg12; do echo "$f: $(grep -v '^W\|^E' $O/$f.out | tr '\n' ' ')"; done
for f in c4r_libpbgpu c4r_libpbgpu_lane12 c4r_libpbgpu_lane15 c4_libpbgpu c4_libpbgpu_lane12 c4_libpbgpu_lane15 c4_mp2 c4_lg11 c4_lg12 c4r_lg11 c4r_lg12; do echo "== $f"; grep -v "^W2026\|^E2026\|^generate\|^per base\|^group" $O/$f.out; done
cat $O/steps.txt
