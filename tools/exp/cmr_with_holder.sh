#!/bin/bash
# create_mega_reads cold runs while another process holds the GPU (an index resident, as
# bench.py's parent does during its create_mega_reads leg): do the runs stall?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=${1:-50000}; R=${2:-8}
D=/tmp/cmr_c2_$N
bash tools/exp/cmr_repeat.sh $N 1 > /dev/null || exit 1
timeout -k 10 200 python -u -c "
import sys, time; sys.path.insert(0, '.')
from pacbio_amd import pbgpu
import os
if os.environ.get('HOLD_GATHER'):
    for ub in (64, 512): pbgpu.measure_gather(0, 64 << 30, unit_bytes=ub)
ix = pbgpu.Index.from_fasta(['$D/sr.fa'], 17, psa_min=13, device=0)
print('holder ready', flush=True)
time.sleep(150)" > gpurun_out/holder.log 2>&1 &
H=$!
for i in $(seq 1 60); do grep -q "holder ready" gpurun_out/holder.log && break; sleep 1; done
PBGPU_DEBUG_STALL=1 bash tools/exp/cmr_repeat.sh $N $R > gpurun_out/holder_rep.log 2>&1
rc=$?
kill $H; wait $H
grep -h "stall" gpurun_out/rep_*.err
sed -e 's/"batches.*"align_s"/"align_s"/' -e 's/"download_s.*//' gpurun_out/holder_rep.log
exit $rc
