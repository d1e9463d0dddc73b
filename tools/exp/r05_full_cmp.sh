# round 5: create_mega_reads device graph == --host-graph on the full C2 (50k) and C4r (20k) read sets
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zy
for w in C4r:20000 C2:50000; do
  n=${w#*:}; w=${w%:*}; D=/tmp/cmr_$w
  timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('$w', seed=42, threads=16, n_pb=$n); ds.write('$D'); ds.close()" || exit 1
  F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
  CMR=pacbio_amd/bin/create_mega_reads
  timeout -k 10 300 $CMR $F -o $D/mr > /dev/null 2>> ${O}_cmp.txt || exit 1
  echo "$w device: $(tail -1 ${O}_cmp.txt | cut -c1-120)" >> ${O}_cmp.txt
  timeout -k 10 600 $CMR $F --host-graph -o $D/mr_host > /dev/null 2>> ${O}_cmp.txt || exit 1
  echo "$w host graph: $(tail -1 ${O}_cmp.txt | cut -c1-120)" >> ${O}_cmp.txt
  if cmp $D/mr $D/mr_host; then echo "$w: device == host graph, $(wc -c < $D/mr) bytes, $(grep -c '^>' $D/mr) reads" >> ${O}_cmp.txt; else echo "$w: DIFFER" >> ${O}_cmp.txt; exit 1; fi
  rm -rf $D
done
grep -E "==|DIFFER" ${O}_cmp.txt
