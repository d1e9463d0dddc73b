#!/bin/bash
# Round 6: create_mega_reads' batch shape on 20k C4r / 50k C2 reads: the run path's 192M-hit
# sub-batch budget (PBGPU_RUN_HIT_BUDGET), aligners per GPU (--streams), batch size, ramp
O=gpurun_out/r06t; mkdir -p gpurun_out/r06t
source tools/r06/lib.sh
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('/tmp/c4r_20k'); ds.close()
ds = Dataset('C2', seed=42, threads=16, n_pb=50000); ds.write('/tmp/c2_50k'); ds.close()"
run() {  # name env... -- extra flags
  local n=$1; shift
  for i in 1 2; do
    step ${W}_${n}_$i 200 env "$@" pacbio_amd/bin/create_mega_reads $F $X -o $D/mr
    echo "$W $n run $i: $(tail -1 $O/${W}_${n}_$i.out | cut -c1-24) $(tail -1 $O/${W}_${n}_$i.out | grep -o '"batches": [0-9]*')"
  done
}
for W in c4r_20k c2_50k; do
D=/tmp/$W
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
X=""
step warm_$W 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
run default A=1
run hb768 PBGPU_RUN_HIT_BUDGET=805306368
run hb768_ramp1 PBGPU_RUN_HIT_BUDGET=805306368 PBGPU_RAMP=1
run ramp1 PBGPU_RAMP=1
X="--streams 1"; run s1_hb1536 PBGPU_RUN_HIT_BUDGET=1610612736
X="--streams 3"; run s3 A=1
X="--batch-bases 32000000"; run b32 A=1
X="--batch-bases 128000000"; run b128_hb1536 PBGPU_RUN_HIT_BUDGET=1610612736
X=""
done
cat $O/steps.txt | grep -v "rc=0"
