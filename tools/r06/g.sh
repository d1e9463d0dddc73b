#!/bin/bash
# Round 6: bucketed grouping of long reads -- parity (edge tests incl. the forced-bucket cases,
# C4r oracle, C4 properties and shards), then C4 / C4r / C2 device legs with and without buckets.
O=gpurun_out/r06g; mkdir -p gpurun_out/r06g
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py
tail -3 $O/tests.out
for b in 1 0; do
  PBGPU_GROUP_BUCKETS=$b step c4_b$b 400 python3 -u tools/prof_c4.py --reads 50000
  grep -v "^W2026\|^E2026" $O/c4_b$b.out
  PBGPU_GROUP_BUCKETS=$b step c4r_b$b 400 python3 -u tools/prof_c4.py --preset C4r --reads 20000
  grep -v "^W2026\|^E2026" $O/c4r_b$b.out
done
step c2 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
cat $O/c2.out
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so step c4p 400 python3 -u tools/prof_c4.py --reads 50000
grep -v "^W2026\|^E2026" $O/c4p.out
step scale 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_gpu_scale.py
tail -3 $O/scale.out
cat $O/steps.txt
