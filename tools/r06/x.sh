#!/bin/bash
# Round 6: graph kernels of 20k C4r reads resident (tools/prof_graph_gpu.py), product vs HEAD
# (libpbgpu_old): rocprofv3 kernel stats and the graph timeline of the timed call
O=gpurun_out/r06x; mkdir -p gpurun_out/r06x
source tools/r06/lib.sh
for v in libpbgpu libpbgpu_old; do
  PBGPU_LIB=pacbio_amd/$v.so step tr_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o g -- python3 -u tools/prof_graph_gpu.py --workload C4r --reads 20000
  head -1 $O/tr_$v.out
  f=$(find $O/tr_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/r06/timeline.py $f --start k_graph_prep --last --top 16 > $O/tl_$v.txt 2>&1
  head -30 $O/tl_$v.txt
done
