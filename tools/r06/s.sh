#!/bin/bash
# Round 6: HIP streams -> hardware queues.  Two aligners make 8 streams (main, group side, two
# graph side streams each) on HIP's 4 queues by default, so streams of different aligners share
# a queue and serialize.  create_mega_reads walls on 20k C4r and 50k C2 reads with
# GPU_MAX_HW_QUEUES 4 (default) / 8 / 12, three runs each after a warm run.
O=gpurun_out/r06s2; mkdir -p gpurun_out/r06s2
source tools/r06/lib.sh
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('/tmp/c4r_20k'); ds.close()
ds = Dataset('C2', seed=42, threads=16, n_pb=50000); ds.write('/tmp/c2_50k'); ds.close()"
for W in c4r_20k c2_50k; do
D=/tmp/$W
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
step warm_$W 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
for q in 4 8 12; do
  for i in 1 2 3; do
    GPU_MAX_HW_QUEUES=$q step ${W}_q${q}_$i 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
    echo "$W queues $q run $i: $(tail -1 $O/${W}_q${q}_$i.out | cut -c1-24)"
  done
done
done
GPU_MAX_HW_QUEUES=8 step trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o c4r -- pacbio_amd/bin/create_mega_reads -s 1M -m 17 --psa-min 13 -k 31 -l /tmp/c4r_20k/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r /tmp/c4r_20k/sr.fa -p /tmp/c4r_20k/pb.fa --timing --devices 0 -o /tmp/c4r_20k/mr
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 tools/r06/timeline.py $f > $O/timeline_q8.txt 2>&1
head -20 $O/timeline_q8.txt
cat $O/steps.txt
