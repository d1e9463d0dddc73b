#!/bin/bash
# Which buffers does a many-batch create_mega_reads run still allocate?  3000 C2 reads,
# --batch-bases 3.2M (>= 12 ramped batches), PBGPU_DEBUG_STALL=2: one line per device
# allocation with the caller's offset in libpbgpu.so (map with nm -C).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
D=$(mktemp -d /tmp/alloc_trace.XXXX)
python -c "
from tools.synth import Dataset
ds = Dataset('C2', seed=42, threads=16, n_pb=${NPB:-3000}); ds.write('$D'); ds.close()" || exit 1
PBGPU_DEBUG_STALL=2 timeout -k 10 300 pacbio_amd/bin/create_mega_reads -s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 \
  --max-count 5000 --stretch-cap 10000 -t 16 --timing --batch-bases ${BB:-3200000} -r $D/sr.fa -p $D/pb.fa -o $D/mr \
  2> gpurun_out/alloc_trace.err
rc=$?
grep -c "pbgpu alloc" gpurun_out/alloc_trace.err; tail -1 gpurun_out/alloc_trace.err
rm -rf $D
exit $rc
