#!/bin/bash
# graph stage ms (tools/prof_graph_gpu.py, C2 50k reads, one aligner) per library variant:
#   bash tools/exp/ab_graph.sh base v1 ...   ("base" = libpbgpu.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  lib=pacbio_amd/libpbgpu_$v.so; [ "$v" = base ] && lib=pacbio_amd/libpbgpu.so
  PBGPU_LIB=$lib timeout -k 10 300 python3 -u tools/prof_graph_gpu.py --reads ${N:-50000} --workload ${WL:-C2} > gpurun_out/abg.log 2>&1 || { tail -5 gpurun_out/abg.log; exit 1; }
  echo "$v $(grep -v '^[EW]20' gpurun_out/abg.log | grep 'graph ')"
done
