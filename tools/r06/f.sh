#!/bin/bash
# Round 6: where C4's group stage goes -- prof_c4 (product and -DPBGPU_PROF), its kernel trace;
# the graph bounds check.
O=gpurun_out/r06f; mkdir -p gpurun_out/r06f
source tools/r06/lib.sh
step prof 400 python3 -u tools/prof_c4.py --reads 50000
cat $O/prof.out
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so step profp 400 python3 -u tools/prof_c4.py --reads 50000
cat $O/profp.out
step trace 400 rocprofv3 --kernel-trace --stats -d $O/trace -o c4 -- python3 -u tools/prof_c4.py --reads 50000
step gcheck 900 bash tools/r06/graph_check.sh $O
cat $O/graph_check.txt
cat $O/steps.txt
