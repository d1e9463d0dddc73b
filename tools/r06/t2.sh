#!/bin/bash
# Round 6: create_mega_reads with fewer, larger batches (no ramp: its output is small, the writer
# is not the bound) on 20k C4r and 50k C2 reads: walls and device peaks
O=gpurun_out/r06t2; mkdir -p gpurun_out/r06t2
source tools/r06/lib.sh
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('/tmp/c4r_20k'); ds.close()
ds = Dataset('C2', seed=42, threads=16, n_pb=50000); ds.write('/tmp/c2_50k'); ds.close()"
run() {  # name: extra flags in X, env in the rest
  local n=$1; shift
  for i in 1 2; do
    step ${W}_${n}_$i 200 env "$@" pacbio_amd/bin/create_mega_reads $F $X -o $D/mr_$n
    echo "$W $n run $i: $(tail -1 $O/${W}_${n}_$i.out | cut -c1-22) $(tail -1 $O/${W}_${n}_$i.out | grep -o '"batches": [0-9]*\|"device_peak_bytes": [0-9]*\|"device_allocs_late": [0-9]*' | tr '\n' ' ')"
  done
}
for W in c4r_20k c2_50k; do
D=/tmp/$W
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
X=""; step warm_$W 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
X=""; run default A=1
X=""; run ramp0 PBGPU_RAMP=0
X="--batch-bases 128000000"; run b128_r0_hb768 PBGPU_RAMP=0 PBGPU_RUN_HIT_BUDGET=805306368
X="--batch-bases 128000000"; run b128_r0_hb1536 PBGPU_RAMP=0 PBGPU_RUN_HIT_BUDGET=1610612736
X="--streams 1 --batch-bases 512000000"; run s1_b512_r0_hb1536 PBGPU_RAMP=0 PBGPU_RUN_HIT_BUDGET=1610612736
X="--batch-bases 256000000"; run b256_r0_hb1536 PBGPU_RAMP=0 PBGPU_RUN_HIT_BUDGET=1610612736
cmp $D/mr_default $D/mr_s1_b512_r0_hb1536 && echo "$W outputs identical"
done
