#!/bin/bash
# rocprofv3 kernel trace of create_mega_reads on C2 reads (device overlap graph).  bash tools/prof_cmr.sh [READS]
set -o pipefail
N=${1:-10000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
D=/tmp/cmr_c2_$N
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.synth import Dataset
ds = Dataset('C2', seed=42, threads=16, n_pb=$N); ds.write('$D'); ds.close()" || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cmr -o run -- pacbio_amd/bin/create_mega_reads $F -o $D/mr > gpurun_out/prof_cmr.log 2>&1 || { tail -20 gpurun_out/prof_cmr.log; exit 1; }
f=$(find gpurun_out/prof_cmr -name "*kernel_stats.csv" | head -1)
if [ -n "$f" ]; then head -25 "$f"; else ls gpurun_out/prof_cmr; fi
