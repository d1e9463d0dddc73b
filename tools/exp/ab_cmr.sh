#!/bin/bash
# create_mega_reads with library variants (pacbio_amd/libpbgpu_<v>.so via LD_LIBRARY_PATH; "base" =
# the product), C2 reads: wall / align / download seconds, output identical to base.
#   bash tools/exp/ab_cmr.sh READS v1 v2 ...
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
for v in base "$@"; do
  L=$PWD/pacbio_amd
  if [ "$v" != base ]; then mkdir -p /tmp/lv_$v && cp pacbio_amd/libpbgpu_$v.so /tmp/lv_$v/libpbgpu.so && L=/tmp/lv_$v; fi
  for rep in 1 2; do
    LD_LIBRARY_PATH=$L timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F -o $D/mr_$v > /dev/null 2> gpurun_out/abcmr_$v.err || { tail -5 gpurun_out/abcmr_$v.err; exit 1; }
    echo "$v: $(tail -1 gpurun_out/abcmr_$v.err | python3 -c 'import json,sys; d=json.load(sys.stdin); print("wall %.3f align %.3f download %.3f graph %.3f" % (d["wall_s"], d["align_s"], d["download_s"], d["graph_s"]))') same=$(cmp -s $D/mr_$v $D/mr_base && echo yes || echo NO)"
  done
done
