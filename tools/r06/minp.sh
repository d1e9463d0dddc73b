#!/bin/bash
# Round 6: with the 8-wave split, bucketing from P >= 1 (PBGPU_GROUP_BUCKET_MINP=1) against 2
O=gpurun_out/r06mp; mkdir -p gpurun_out/r06mp
source tools/r06/lib.sh
for rep in 1 2; do
for m in 2 1; do
  PBGPU_GROUP_BUCKET_MINP=$m step c4_${m}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  PBGPU_GROUP_BUCKET_MINP=$m step c4r_${m}_$rep 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  PBGPU_GROUP_BUCKET_MINP=$m step c2_${m}_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  for w in c4 c4r; do echo "$w minp=$m $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/${w}_${m}_$rep.out | head -2 | tr '\n' ' ' | cut -c1-230)"; done
  echo "c2 minp=$m $rep: $(grep 'stages ms' $O/c2_${m}_$rep.out | cut -c1-200)"
done
done
