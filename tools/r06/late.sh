#!/bin/bash
# Round 6: which device allocations happen after a worker's first batch in
# test_no_device_allocation_after_first_batch's run (3000 C2 reads, 3.2-Mbase batches)
O=gpurun_out/r06late; mkdir -p gpurun_out/r06late
source tools/r06/lib.sh
D=/tmp/c2_3k
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C2', seed=42, threads=16, n_pb=3000); ds.write('$D'); ds.close()"
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 --timing -r $D/sr.fa -p $D/pb.fa --batch-bases 3200000"
PBGPU_DEBUG_STALL=2 PBGPU_TIMELINE=1 step allocs 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
tail -1 $O/allocs.out
