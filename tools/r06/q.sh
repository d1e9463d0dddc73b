#!/bin/bash
# Round 6: kernel timeline of create_mega_reads on 20k C4r reads (bench's c4r flags), one warm run
# first; the window from the first k_seed, busy fraction, idle gaps, kernel totals (tools/r06/timeline.py)
O=gpurun_out/r06q; mkdir -p gpurun_out/r06q
source tools/r06/lib.sh
D=/tmp/c4r_20k
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('$D'); ds.close()"
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
step warm 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
tail -1 $O/warm.out
step run2 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
tail -1 $O/run2.out
step trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o c4r -- pacbio_amd/bin/create_mega_reads $F -o $D/mr
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 tools/r06/timeline.py $f > $O/timeline.txt 2>&1
cat $O/timeline.txt | head -70
cat $O/steps.txt
