#!/bin/bash
# create_mega_reads on C4r reads (C4's repeat model and read lengths): 2 cold runs, --timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=${1:-20000}; D=/tmp/cmr_c4r_$N
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C4r', seed=42, threads=16, n_pb=$N); ds.write('$D'); ds.close()" || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
for i in 1 2; do
  timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F -o $D/mr > /dev/null 2> gpurun_out/c4r_cmr_$i.err || { tail -5 gpurun_out/c4r_cmr_$i.err; exit 1; }
  echo "run $i: $(tail -1 gpurun_out/c4r_cmr_$i.err)"
done
