# round 5: create_mega_reads batch ramp and batch size on C4r / C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zj
for w in C4r:20000 C2:50000; do
  n=${w#*:}; w=${w%:*}; D=/tmp/cmr_$w
  timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('$w', seed=42, threads=16, n_pb=$n); ds.write('$D'); ds.close()" || exit 1
  F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
  CMR=pacbio_amd/bin/create_mega_reads
  timeout -k 10 120 $CMR $F -o $D/mr > /dev/null 2> /dev/null || exit 1
  for v in "3 64M" "1 64M" "0 64M" "2 96M" "1 96M" "3 128M" "1 128M" "3 48M"; do
    set -- $v
    for i in 1 2; do
      echo "== $w ramp $1 batch $2" >> ${O}_ramp.txt
      PBGPU_RAMP=$1 timeout -k 10 120 $CMR $F --batch-bases $2 -o $D/mr > /dev/null 2>> ${O}_ramp.txt || exit 1
    done
  done
  rm -rf $D
done
