# round 5: C4r create_mega_reads -- which buffers grow late (PBGPU_DEBUG_STALL=2), a kernel trace, group table phases
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05o
w=C4r; n=20000; D=/tmp/cmr_$w
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('$w', seed=42, threads=16, n_pb=$n); ds.write('$D'); ds.close()" || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
PBGPU_DEBUG_STALL=2 PBGPU_TIMELINE=1 timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F -o $D/mr > /dev/null 2> ${O}_alloc.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05o_prof -o c4r -- pacbio_amd/bin/create_mega_reads $F -o $D/mr > /dev/null 2> ${O}_prof.err || exit 1
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_lis.py --workload C4r --reads 20000 > ${O}_group_prof.txt 2>&1
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python -u tools/prof_graph_gpu.py --workload C4r --reads 20000 > ${O}_graph_prof.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_mega_reads.py::test_graph_ties_equal_implied_starts" > ${O}_tests.log 2>&1
