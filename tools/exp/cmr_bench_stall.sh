#!/bin/bash
# bench.py's create_mega_reads leg (children of the bench process) with stall reports per run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-g}; R=${2:-8}; shift 2
timeout -k 10 500 python -u bench.py --steps 1 --warmup 0 --device-steps 1 --parts 0 --cmr-steps $R --no-cpu-baseline --skip-default-leg "$@" > gpurun_out/cmr_stall_$TAG.json 2> gpurun_out/cmr_stall_$TAG.err || { tail -5 gpurun_out/cmr_stall_$TAG.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/cmr_stall_$TAG.json'))
print('cmr', d['value_create_mega_reads']/1e9, d['create_mega_reads_walls_s'])
for r in d['create_mega_reads_runs']: print(r['wall_s'], r['align_s'], r.get('alloc_s'), r.get('device_alloc_bytes'), r.get('device_allocs'), r['stalls'])"
