#!/bin/bash
# Round 6: the grouping's prediction scale (PBGPU_GROUP_PRED_SCALE 1.0 / 1.3 / 1.6: reads near
# the 4-wave tier's fill go to the bucketed path instead of overflowing into a later round)
O=gpurun_out/r06ps; mkdir -p gpurun_out/r06ps
source tools/r06/lib.sh
for rep in 1 2; do
for s in 1.0 1.3 1.6; do
  n=${s/./_}
  PBGPU_GROUP_PRED_SCALE=$s step c4_${n}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  echo "c4 scale=$s $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base' $O/c4_${n}_$rep.out | head -3 | tr '\n' ' ' | cut -c1-330)"
done
done
for s in 1.0 1.3 1.6; do
  n=${s/./_}
  PBGPU_GROUP_PRED_SCALE=$s step c4r_$n 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  PBGPU_GROUP_PRED_SCALE=$s step c2_$n 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  echo "c4r scale=$s: $(grep -v '^W2026\|^E2026\|^generate\|^per base' $O/c4r_$n.out | head -3 | tr '\n' ' ' | cut -c1-330)"
  echo "c2 scale=$s: $(grep 'stages ms\|tier0' $O/c2_$n.out | tr '\n' ' ' | cut -c1-260)"
done
