#!/bin/bash
# create_mega_reads on C2 reads with extra option sets (the product library): wall / align /
# graph seconds per set, output identical to the first set's.
#   bash tools/exp/ab_cmr_opts.sh READS "--streams 2" "--streams 3" ...
set -o pipefail
N=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
D=/tmp/cmr_c2_$N
[ -f $D/pb.fa ] || timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C2', seed=42, threads=16, n_pb=$N); ds.write('$D'); ds.close()" || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
i=0
for o in "$@"; do
  for rep in 1 2; do
    timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F $o -o $D/mr_$i > /dev/null 2> gpurun_out/abopt_$i.err || { tail -5 gpurun_out/abopt_$i.err; exit 1; }
    echo "[$o]: $(tail -1 gpurun_out/abopt_$i.err | python3 -c 'import json,sys; d=json.load(sys.stdin); print("wall %.3f align %.3f download %.3f graph %.3f batches %d" % (d["wall_s"], d["align_s"], d["download_s"], d["graph_s"], d["batches"]))') same=$(cmp -s $D/mr_$i $D/mr_0 && echo yes || echo NO)"
  done
  i=$((i+1))
done
