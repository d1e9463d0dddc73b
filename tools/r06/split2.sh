#!/bin/bash
# Round 6: the split launch's block size (PBGPU_SPLIT_BLOCK 128 / 256 (default) / 512): C4, C4r; parity
O=gpurun_out/r06sp2; mkdir -p gpurun_out/r06sp2
source tools/r06/lib.sh
for b in 128 512; do
  PBGPU_SPLIT_BLOCK=$b step tests_$b 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py -k bucketed
  echo "tests split=$b: $(tail -1 $O/tests_$b.out)"
done
for rep in 1 2; do
for b in 128 256 512; do
  PBGPU_SPLIT_BLOCK=$b step c4_${b}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  echo "c4 split=$b $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/c4_${b}_$rep.out | head -2 | tr '\n' ' ' | cut -c1-230)"
done
done
for b in 128 256 512; do
  PBGPU_SPLIT_BLOCK=$b step c4r_$b 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  echo "c4r split=$b: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/c4r_$b.out | head -2 | tr '\n' ' ' | cut -c1-230)"
done
