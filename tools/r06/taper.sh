#!/bin/bash
# Round 6: the end-of-input taper (the input's last < W full batches split evenly over the W
# aligners) against PBGPU_TAPER=0: create_mega_reads on 20k C4r / 50k C2 reads, the bench's
# coords-out leg; the CLI tests
O=gpurun_out/r06tp; mkdir -p gpurun_out/r06tp
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_mega_reads.py tests/test_gpu_streams.py tests/test_gpu_format.py
tail -1 $O/tests.out
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('/tmp/c4r_20k'); ds.close()
ds = Dataset('C2', seed=42, threads=16, n_pb=50000); ds.write('/tmp/c2_50k'); ds.close()"
for W in c4r_20k c2_50k; do
D=/tmp/$W
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
step warm_$W 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr
for i in 1 2 3; do
  for t in 1 0; do
    PBGPU_TAPER=$t step ${W}_t${t}_$i 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr_t$t
    echo "$W taper=$t $i: $(tail -1 $O/${W}_t${t}_$i.out | cut -c1-22) $(tail -1 $O/${W}_t${t}_$i.out | grep -o '"batches": [0-9]*\|"device_allocs_late": [0-9]*' | tr '\n' ' ')"
  done
done
cmp $D/mr_t1 $D/mr_t0 && echo "$W outputs identical"
done
for t in 1 0; do
  PBGPU_TAPER=$t step bench_t$t 400 python3 -u bench.py --c4r-reads 0 --c3-reads 0 --c4-reads 0 --no-cpu-baseline --parts 0 --cmr-steps 0
  echo "bench taper=$t: $(grep '^{"metric"' $O/bench_t$t.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
