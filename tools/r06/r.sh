#!/bin/bash
# Round 6: what bounds k_graph_relax_big on C4r: phase ticks (prof build) and the edge-block
# prefetch distance (PBGPU_RELAX_PF 3 / 6 product / 12), graph stage of 20k C4r reads resident and
# create_mega_reads walls with each library
O=gpurun_out/r06r; mkdir -p gpurun_out/r06r
source tools/r06/lib.sh
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so step prof 300 python3 -u tools/prof_graph_gpu.py --workload C4r --reads 20000
cat $O/prof.out | grep -v "^W2026\|^E2026"
for v in libpbgpu libpbgpu_pf3 libpbgpu_pf12; do
  PBGPU_LIB=pacbio_amd/$v.so step g_$v 300 python3 -u tools/prof_graph_gpu.py --workload C4r --reads 20000
  head -1 $O/g_$v.out
done
D=/tmp/c4r_20k
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('$D'); ds.close()"
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
for v in libpbgpu_pf3 libpbgpu_pf12 libpbgpu; do
  mkdir -p /tmp/lib_$v; cp pacbio_amd/$v.so /tmp/lib_$v/libpbgpu.so
  for i in 1 2 3; do
    LD_LIBRARY_PATH=/tmp/lib_$v step cmr_${v}_$i 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
    echo "cmr $v $i: $(tail -1 $O/cmr_${v}_$i.out | cut -c1-60)"
  done
done
cat $O/steps.txt
