#!/bin/bash
# Round 6: SrMeta lines for k_coords' prologue (variant libpbgpu_meta) against the product; bucketing
# every read past the small tier (PBGPU_GROUP_BUCKET_MINP=1); parity of the variant.
O=gpurun_out/r06p; mkdir -p gpurun_out/r06p
source tools/r06/lib.sh
PBGPU_LIB=pacbio_amd/libpbgpu_meta.so step tests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fine_details.py
tail -2 $O/tests.out
for rep in 1 2; do
for v in libpbgpu libpbgpu_meta; do
  PBGPU_LIB=pacbio_amd/$v.so step c2_${v}_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_LIB=pacbio_amd/$v.so step c4_${v}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
done
done
PBGPU_LIB=pacbio_amd/libpbgpu_meta.so PBGPU_GROUP_BUCKET_MINP=1 step c4_mp1 400 python3 -u tools/prof_c4.py --reads 50000
PBGPU_LIB=pacbio_amd/libpbgpu_meta.so PBGPU_GROUP_BUCKET_MINP=1 step c4r_mp1 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
PBGPU_LIB=pacbio_amd/libpbgpu_meta.so step c4r_meta 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
PBGPU_LIB=pacbio_amd/libpbgpu_meta.so PBGPU_GROUP_BUCKET_MINP=1 step c2_mp1 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
for f in c2_libpbgpu_1 c2_libpbgpu_meta_1 c2_libpbgpu_2 c2_libpbgpu_meta_2 c2_mp1; do echo "$f: $(grep -v '^W\|^E' $O/$f.out | tr '\n' ' ')"; done
for f in c4_libpbgpu_1 c4_libpbgpu_meta_1 c4_libpbgpu_2 c4_libpbgpu_meta_2 c4_mp1 c4r_meta c4r_mp1; do echo "== $f: $(grep -v "^W2026\|^E2026\|^generate\|^per base\|^group" $O/$f.out | tr '\n' ' ')"; done
cat $O/steps.txt
