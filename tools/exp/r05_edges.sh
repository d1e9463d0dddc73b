# round 5: k_graph_edges' block fast-forward -- parity (device == host graph), scan counts, walls; group table phases
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05l
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C4r --reads 20000 > ${O}_graph_prof.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C4r --reads 20000 > ${O}_graph.txt 2>&1 || exit 1
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_lis.py --workload C4r --reads 20000 > ${O}_group_prof.txt 2>&1 || exit 1
w=C4r; n=20000; D=/tmp/cmr_$w
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('$w', seed=42, threads=16, n_pb=$n); ds.write('$D'); ds.close()" || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
for i in 1 2; do
  PBGPU_DEBUG_STALL=1 timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F -o $D/mr > /dev/null 2> ${O}_cmr_${w}_$i.err || { tail -5 ${O}_cmr_${w}_$i.err; exit 1; }
  echo "$w run $i: $(tail -1 ${O}_cmr_${w}_$i.err)" >> ${O}_cmr.txt
done
timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F --host-graph -o $D/mr_host > /dev/null 2>&1 || exit 1
cmp $D/mr $D/mr_host && echo "$w device == host graph" >> ${O}_cmr.txt
