# round 5: create_mega_reads working set by buffer (PBGPU_DEBUG_BUFFERS=1) on C2 (50k) and C4r (20k),
# the late-allocation test, and a kernel trace of one C4r run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_mega_reads.py::test_no_device_allocation_after_first_batch" > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
for W in C2:50000 C4r:20000; do
  w=${W%%:*}; n=${W##*:}; D=/tmp/cmr_$w
  timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('$w', seed=42, threads=16, n_pb=$n); ds.write('$D'); ds.close()" || exit 1
  F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
  for i in 1 2 3; do
    PBGPU_DEBUG_BUFFERS=1 PBGPU_DEBUG_STALL=1 timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F -o $D/mr > /dev/null 2> ${O}_cmr_${w}_$i.err || { tail -5 ${O}_cmr_${w}_$i.err; exit 1; }
    echo "$w run $i: $(tail -1 ${O}_cmr_${w}_$i.err)" >> ${O}_cmr.txt
  done
done
D=/tmp/cmr_C4r
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05e_prof -o c4r -- pacbio_amd/bin/create_mega_reads -s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing -o $D/mr > /dev/null 2> ${O}_prof.err
