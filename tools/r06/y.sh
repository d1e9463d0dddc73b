#!/bin/bash
# Round 6: k_graph_relax_big union-find tiers up to 32768 records in LDS, the long tiers spread
# over the side streams: graph parity, resident graph kernels (20k C4r) and create_mega_reads
# walls against HEAD (libpbgpu_old)
O=gpurun_out/r06y; mkdir -p gpurun_out/r06y
source tools/r06/lib.sh
step tests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_mega_reads.py
tail -1 $O/tests.out
for v in libpbgpu libpbgpu_old; do
  PBGPU_LIB=pacbio_amd/$v.so step tr_$v 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o g -- python3 -u tools/prof_graph_gpu.py --workload C4r --reads 20000
  f=$(find $O/tr_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/r06/timeline.py $f --start k_graph_prep --last --top 12 > $O/tl_$v.txt 2>&1
  echo "== $v: $(grep 'align_resident' $O/tr_$v.out | tail -1)"; head -22 $O/tl_$v.txt
done
step gen 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=20000); ds.write('/tmp/c4r_20k'); ds.close()"
D=/tmp/c4r_20k
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing --devices 0"
for v in libpbgpu libpbgpu_old; do
  mkdir -p /tmp/lib_$v; cp pacbio_amd/$v.so /tmp/lib_$v/libpbgpu.so
  LD_LIBRARY_PATH=/tmp/lib_$v step warm_$v 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr_$v
done
for i in 1 2 3 4; do
  for v in libpbgpu libpbgpu_old; do
    LD_LIBRARY_PATH=/tmp/lib_$v step c4r_${v}_$i 200 pacbio_amd/bin/create_mega_reads $F -o $D/mr_$v
    echo "c4r $v $i: $(tail -1 $O/c4r_${v}_$i.out | cut -c1-24)"
  done
done
cmp $D/mr_libpbgpu $D/mr_libpbgpu_old && echo "outputs identical"
