#!/bin/bash
# k_graph_relax phase ticks (PBGPU_PROF library), then the create_mega_reads leg's per-run stages
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-g}
PBGPU_LIB=pacbio_amd/libpbgpu_prof.so timeout -k 10 300 python3 -u tools/prof_graph_gpu.py --reads 50000 > gpurun_out/relax_prof_$TAG.log 2>&1 || { tail -20 gpurun_out/relax_prof_$TAG.log; exit 1; }
grep -v "^[EW]20" gpurun_out/relax_prof_$TAG.log | tail -12
timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --device-steps 1 --parts 0 --cmr-steps 5 --no-cpu-baseline --no-brand --skip-default-leg > gpurun_out/cmr_runs_$TAG.json 2> gpurun_out/cmr_runs_$TAG.err || { tail -5 gpurun_out/cmr_runs_$TAG.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/cmr_runs_$TAG.json'))
print('cmr', d['value_create_mega_reads']/1e9, d['create_mega_reads_walls_s'])
for r in d['create_mega_reads_runs']: print({k: v for k, v in r.items() if k.endswith('_s')})"
