#!/bin/bash
# Round 6: the 4-B super-read side array (PBGPU_OCC_SR=1: k_group's counting passes read 4 B an
# occurrence from a packed array instead of the 8-B words' lines) on C4 (49 GB more HBM) and C4r
O=gpurun_out/r06osr; mkdir -p gpurun_out/r06osr
source tools/r06/lib.sh
for rep in 1 2; do
for v in 0 1; do
  PBGPU_OCC_SR=$v step c4_${v}_${rep} 400 python3 -u tools/prof_c4.py --reads 50000
  PBGPU_OCC_SR=$v step c4r_${v}_${rep} 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  for w in c4 c4r; do echo "$w occ_sr=$v $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/${w}_${v}_${rep}.out | head -2 | tr '\n' ' ' | cut -c1-260)"; done
done
done
