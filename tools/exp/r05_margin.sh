# round 5: learnt partition margin of the 8192-slot group tier -- group tests, stages, cmr C4r + trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zi
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_edge.py tests/test_gpu_parity.py tests/test_gpu_configs.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for wl in "C2 50000" "C4r 20000"; do
  set -- $wl
  timeout -k 10 300 python -u tools/prof_lis.py --workload $1 --reads $2 >> ${O}_stages.txt 2>&1 || exit 1
done
grep stages ${O}_stages.txt
for w in C4r:20000 C2:50000; do
  n=${w#*:}; w=${w%:*}; D=/tmp/cmr_$w
  timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('$w', seed=42, threads=16, n_pb=$n); ds.write('$D'); ds.close()" || exit 1
  F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
  CMR=pacbio_amd/bin/create_mega_reads
  timeout -k 10 120 $CMR $F -o $D/mr > /dev/null 2> /dev/null || exit 1
  for i in 1 2 3; do
    echo "== $w run $i" >> ${O}_cmr.txt
    timeout -k 10 120 $CMR $F -o $D/mr > /dev/null 2>> ${O}_cmr.txt || exit 1
  done
  if [ $w = C4r ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05zi_prof -o s1 -- $CMR $F --streams 1 -o $D/mr > /dev/null 2> ${O}_prof.err || exit 1
  fi
  rm -rf $D
done
