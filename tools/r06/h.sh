#!/bin/bash
# Round 6: bucketed grouping -- edge tests; C2 A/B on one box (this tree, buckets on / off, and
# the library of the previous commit); C4 device path; graph bounds check.
O=gpurun_out/r06h; mkdir -p gpurun_out/r06h
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_edge.py
tail -3 $O/tests.out
for rep in 1 2; do
  step c2_cur_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_GROUP_BUCKETS=0 step c2_nob_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  PBGPU_LIB=pacbio_amd/libpbgpu_head.so step c2_head_$rep 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
done
for f in c2_cur_1 c2_nob_1 c2_head_1 c2_cur_2 c2_nob_2 c2_head_2; do echo "$f: $(grep -v '^W\|^E' $O/$f.out | tr '\n' ' ')"; done
step c4 400 python3 -u tools/prof_c4.py --reads 50000
grep -v "^W2026\|^E2026" $O/c4.out
step gcheck 900 bash tools/r06/graph_check.sh $O
cat $O/graph_check.txt
cat $O/steps.txt
