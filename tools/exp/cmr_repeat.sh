#!/bin/bash
# create_mega_reads on C2 reads, R cold runs with the product flags: every run's --timing line.
#   bash tools/exp/cmr_repeat.sh READS R [extra flags]
set -o pipefail
N=$1; R=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
D=/tmp/cmr_c2_$N
[ -f $D/pb.fa ] || timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C2', seed=42, threads=16, n_pb=$N); ds.write('$D'); ds.close()" || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
for i in $(seq 1 $R); do
  [ -n "$PAUSE" ] && [ $i -gt 1 ] && sleep $PAUSE
  s=$(date +%s.%N)
  timeout -k 10 120 pacbio_amd/bin/create_mega_reads $F "$@" -o $D/mr > /dev/null 2> gpurun_out/rep_$i.err || { tail -5 gpurun_out/rep_$i.err; exit 1; }
  e=$(date +%s.%N)
  echo "run $i: $(tail -1 gpurun_out/rep_$i.err)"
done
