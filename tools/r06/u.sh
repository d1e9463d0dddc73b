#!/bin/bash
# Round 6: which buffers create_mega_reads still allocates after a worker's first batch on 50k C2
# reads (PBGPU_DEBUG_STALL=2: every device allocation with its caller; PBGPU_TIMELINE=1: batches)
O=gpurun_out/r06u; mkdir -p gpurun_out/r06u
source tools/r06/lib.sh
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C2', seed=42, threads=16, n_pb=50000); ds.write('/tmp/c2_50k'); ds.close()"
D=/tmp/c2_50k
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
PBGPU_DEBUG_STALL=2 PBGPU_TIMELINE=1 step allocs 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
grep -c "pbgpu alloc" $O/allocs.out
tail -1 $O/allocs.out
