#!/bin/bash
# Round 6, with the 8-wave split and P >= 1: bucket items' table size (PBGPU_GROUP_BUCKET_LOG2 10
# vs 11) and partition margin (PBGPU_GROUP_BUCKET_MARGIN 1.25 / 1.5 / 2.0) on C4 and C4r
O=gpurun_out/r06bk; mkdir -p gpurun_out/r06bk
source tools/r06/lib.sh
for rep in 1 2; do
for cfg in "PBGPU_GROUP_BUCKET_LOG2=11" "PBGPU_GROUP_BUCKET_LOG2=10" "PBGPU_GROUP_BUCKET_MARGIN=1.25" "PBGPU_GROUP_BUCKET_MARGIN=2.0"; do
  n=$(echo $cfg | tr '=.' '__')
  eval "$cfg step c4_${n}_$rep 400 python3 -u tools/prof_c4.py --reads 50000"
  echo "c4 $cfg $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base' $O/c4_${n}_$rep.out | head -3 | tr '\n' ' ' | cut -c1-330)"
done
done
for cfg in "PBGPU_GROUP_BUCKET_LOG2=11" "PBGPU_GROUP_BUCKET_LOG2=10"; do
  n=$(echo $cfg | tr '=.' '__')
  eval "$cfg step c4r_$n 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000"
  echo "c4r $cfg: $(grep -v '^W2026\|^E2026\|^generate\|^per base' $O/c4r_$n.out | head -3 | tr '\n' ' ' | cut -c1-330)"
done
