#!/bin/bash
# Round 6: the bucket items in 8-wave blocks (PBGPU_BUCKET_BLOCK=512) against 4-wave: C4, C4r; parity
O=gpurun_out/r06bb; mkdir -p gpurun_out/r06bb
source tools/r06/lib.sh
PBGPU_BUCKET_BLOCK=512 step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py
echo "tests 512: $(tail -1 $O/tests.out)"
for rep in 1 2; do
for b in 256 512; do
  PBGPU_BUCKET_BLOCK=$b step c4_${b}_$rep 400 python3 -u tools/prof_c4.py --reads 50000
  PBGPU_BUCKET_BLOCK=$b step c4r_${b}_$rep 300 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  for w in c4 c4r; do echo "$w bucket=$b $rep: $(grep -v '^W2026\|^E2026\|^generate\|^per base\|^group' $O/${w}_${b}_$rep.out | head -2 | tr '\n' ' ' | cut -c1-230)"; done
done
done
