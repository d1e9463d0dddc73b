#!/bin/bash
# Round 6: bucket items on a 1024-slot table (PBGPU_GROUP_BUCKET_LOG2=10: twice the partitions,
# 19 KB of LDS a block, 8 blocks a CU) against 2048 slots: C4, C4r, parity
O=gpurun_out/r06lg; mkdir -p gpurun_out/r06lg
source tools/r06/lib.sh
PBGPU_GROUP_BUCKET_LOG2=10 step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py
echo "tests lg10: $(tail -1 $O/tests.out)"
for rep in 1 2; do
for l in 11 10; do
  PBGPU_GROUP_BUCKET_LOG2=$l step c4_${l}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  echo "c4 lg$l $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base' $O/c4_${l}_$rep.out | head -3 | tr '\n' ' ' | cut -c1-300)"
done
done
for l in 11 10; do
  PBGPU_GROUP_BUCKET_LOG2=$l step c4r_$l 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  echo "c4r lg$l: $(grep -v '^W2026\|^E2026\|^generate\|^per base' $O/c4r_$l.out | head -3 | tr '\n' ' ' | cut -c1-300)"
done
