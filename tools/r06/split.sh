#!/bin/bash
# Round 6: the bucket split launch in 4-wave blocks (PBGPU_SPLIT_BLOCK=256; its LDS now sized by
# the launch's largest P) against 16-wave blocks: group stage on C4 / C4r / C2, parity
O=gpurun_out/r06sp; mkdir -p gpurun_out/r06sp
source tools/r06/lib.sh
PBGPU_SPLIT_BLOCK=256 step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py
tail -1 $O/tests.out
for rep in 1 2; do
for b in 1024 256; do
  PBGPU_SPLIT_BLOCK=$b step c4_${b}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  PBGPU_SPLIT_BLOCK=$b step c4r_${b}_$rep 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  for w in c4 c4r; do echo "$w split=$b $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/${w}_${b}_$rep.out | head -2 | tr '\n' ' ' | cut -c1-230)"; done
done
done
PBGPU_SPLIT_BLOCK=256 step c2_256 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
step c2_1024 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
for b in 1024 256; do echo "c2 split=$b: $(grep 'stages ms' $O/c2_$b.out | cut -c1-200)"; done
