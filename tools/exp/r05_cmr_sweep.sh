# round 5: why create_mega_reads on C4r spends 4x the resident call's group time -- streams,
# batch size and hit budget varied; a kernel trace of the one-stream run; long-strand LIS tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05q
w=C4r; n=20000; D=/tmp/cmr_$w
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('$w', seed=42, threads=16, n_pb=$n); ds.write('$D'); ds.close()" || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
CMR=pacbio_amd/bin/create_mega_reads
timeout -k 10 120 $CMR $F -o $D/mr > /dev/null 2> /dev/null || exit 1   # warm (page cache)
for v in "" "--streams 1" "--batch-bases 300M" "--batch-bases 300M --streams 1" "--batch-bases 16M"; do
  echo "== $v" >> ${O}_sweep.txt
  timeout -k 10 120 $CMR $F $v -o $D/mr > /dev/null 2>> ${O}_sweep.txt || exit 1
done
for b in 400000000 1000000000; do
  echo "== PBGPU_RUN_HIT_BUDGET=$b" >> ${O}_sweep.txt
  PBGPU_RUN_HIT_BUDGET=$b timeout -k 10 120 $CMR $F -o $D/mr > /dev/null 2>> ${O}_sweep.txt || exit 1
  echo "== PBGPU_RUN_HIT_BUDGET=$b --streams 1" >> ${O}_sweep.txt
  PBGPU_RUN_HIT_BUDGET=$b timeout -k 10 120 $CMR $F --streams 1 -o $D/mr > /dev/null 2>> ${O}_sweep.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05q_prof -o s1 -- $CMR $F --streams 1 -o $D/mr > /dev/null 2> ${O}_prof.err || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_edge.py::test_long_strands" tests/test_gpu_mega_reads.py > ${O}_tests.log 2>&1
tail -1 ${O}_tests.log
for e in 0 1; do
  echo "== PBGPU_LISW_SHORT=$e" >> gpurun_out/r05p_lisw.txt
  PBGPU_LISW_SHORT=$e timeout -k 10 300 python -u tools/prof_lis.py --workload C2 --reads 50000 >> gpurun_out/r05p_lisw.txt 2>&1 || exit 1
  PBGPU_LISW_SHORT=$e timeout -k 10 300 python -u tools/prof_lis.py --workload C4r --reads 20000 >> gpurun_out/r05p_lisw.txt 2>&1 || exit 1
done
