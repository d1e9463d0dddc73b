#!/bin/bash
# kernel trace (with memory copies) of one create_mega_reads run on 50k C2 reads:
# where does the first batches' time go?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=50000; D=/tmp/cmr_c2_$N
bash tools/exp/cmr_repeat.sh $N 1 > /dev/null || exit 1
F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 -r $D/sr.fa -p $D/pb.fa --timing"
O=gpurun_out/cmr_kt; rm -rf $O; mkdir -p $O
PBGPU_TIMELINE=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O -o run -- pacbio_amd/bin/create_mega_reads $F -o $D/mr > $O/out.log 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
grep "pbgpu tl\|wall_s" $O/err.log | tail -40 > $O/timeline.txt
ls $O
