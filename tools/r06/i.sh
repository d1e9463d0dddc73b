#!/bin/bash
# Round 6: the split on a side stream -- edge tests; C2 A/B (buckets on / off, twice); C4 and
# C4r device paths with the phase profile and a kernel trace.
O=gpurun_out/r06i; mkdir -p gpurun_out/r06i
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py tests/test_gpu_configs.py
tail -3 $O/tests.out
for rep in 1 2; do
  step c2_cur_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_GROUP_BUCKETS=0 step c2_nob_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
done
for f in c2_cur_1 c2_nob_1 c2_cur_2 c2_nob_2; do echo "$f: $(grep -v '^W\|^E' $O/$f.out | tr '\n' ' ')"; done
step c4 400 python3 -u tools/prof_c4.py --reads 50000
grep -v "^W2026\|^E2026" $O/c4.out
step c4r 400 python3 -u tools/prof_c4.py --preset C4r --reads 20000
grep -v "^W2026\|^E2026" $O/c4r.out
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so step c4p 400 python3 -u tools/prof_c4.py --reads 50000
grep -v "^W2026\|^E2026" $O/c4p.out
step trace 400 rocprofv3 --kernel-trace --stats -d $O/trace -o c4 -- python3 -u tools/prof_c4.py --reads 50000
cat $O/steps.txt
