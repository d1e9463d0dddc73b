#!/bin/bash
# Round 6: k_graph_relax_big with its union-find in LDS (tiers 4096 / 16384), and (root-encoded, 2 B a node, tiers 4096 / 8192 / 16384) against HEAD (variant libpbgpu_old)
# per-chunk workgroup fence (variant libpbgpu_old): graph parity, phase ticks, graph stage
# of 20k C4r reads resident, create_mega_reads walls on C4r and C2
O=gpurun_out/r06w; mkdir -p gpurun_out/r06w
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_mega_reads.py
tail -2 $O/tests.out
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so step prof 300 python3 -u tools/prof_graph_gpu.py --workload C4r --reads 20000
grep "relax" $O/prof.out
for v in libpbgpu libpbgpu_old; do
  PBGPU_LIB=pacbio_amd/$v.so step g_$v 300 python3 -u tools/prof_graph_gpu.py --workload C4r --reads 20000
  echo "$v: $(head -1 $O/g_$v.out)"
done
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('/tmp/c4r_20k'); ds.close()
ds = Dataset('C2', seed=42, threads=16, n_pb=50000); ds.write('/tmp/c2_50k'); ds.close()"
for W in c4r_20k c2_50k; do
D=/tmp/$W
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
for v in libpbgpu libpbgpu_old; do
  mkdir -p /tmp/lib_$v; cp pacbio_amd/$v.so /tmp/lib_$v/libpbgpu.so
  LD_LIBRARY_PATH=/tmp/lib_$v step warm_${W}_$v 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr_$v
  for i in 1 2 3; do
    LD_LIBRARY_PATH=/tmp/lib_$v step ${W}_${v}_$i 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr_$v
    echo "$W $v $i: $(tail -1 $O/${W}_${v}_$i.out | cut -c1-24) late $(tail -1 $O/${W}_${v}_$i.out | grep -o '"device_allocs_late": [0-9]*')"
  done
done
cmp $D/mr_libpbgpu $D/mr_libpbgpu_old && echo "$W outputs identical"
done
cat $O/steps.txt
step trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o c4r -- pacbio_amd/bin/create_mega_reads -s 1M -m 17 --psa-min 13 -k 31 -l /tmp/c4r_20k/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r /tmp/c4r_20k/sr.fa -p /tmp/c4r_20k/pb.fa --timing --devices 0 -o /tmp/c4r_20k/mr
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 tools/r06/timeline.py $f > $O/timeline.txt 2>&1
head -30 $O/timeline.txt
