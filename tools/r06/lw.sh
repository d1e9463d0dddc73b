#!/bin/bash
# Round 6: k_lis_w<255, 8> occupancy -- waves per SIMD asked of the compiler (PBGPU_LISW_WAVES 7 / 8:
# 72 / 64 VGPRs with 4 / 13 spilled, against 79 VGPRs = 6 waves): LIS stage on C2 and C4
O=gpurun_out/r06lw; mkdir -p gpurun_out/r06lw
source tools/r06/lib.sh
for rep in 1 2; do
for v in libpbgpu libpbgpu_lw7 libpbgpu_lw8; do
  PBGPU_LIB=pacbio_amd/$v.so step c2_${v}_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_LIB=pacbio_amd/$v.so step c4_${v}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  for w in c2 c4; do echo "$w $v $rep: $(grep 'stages ms' $O/${w}_${v}_$rep.out | head -1 | cut -c1-200)"; done
done
done
PBGPU_LIB=pacbio_amd/libpbgpu_lw7.so step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py
tail -1 $O/tests.out
# SQ counters of the C4 LIS kernels (register LIS, wave LIS, permutation)
step sq_c4 600 bash tools/pmc_sq_any.sh "k_lis_tiny|k_lis_w|k_len_perm|k_init_slen" $O/sq_c4 -- python3 tools/prof_c4.py --reads 50000
grep -v "^W2026\|^E2026" $O/sq_c4.out | tail -40
