#!/bin/bash
# device-leg stage times (bench.py's device leg, C2) per library variant: bash tools/exp/ab_dev.sh base v1 ...
# ("base" = libpbgpu.so); interleave variants to see the box's run-to-run spread
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  lib=pacbio_amd/libpbgpu_$v.so; [ "$v" = base ] && lib=pacbio_amd/libpbgpu.so
  PBGPU_LIB=$lib timeout -k 10 400 python bench.py --steps 1 --warmup 0 --device-steps 3 --parts 0 --cmr-steps 0 --no-cpu-baseline --skip-default-leg --no-brand > gpurun_out/abd.json 2> gpurun_out/abd.err || { tail -5 gpurun_out/abd.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/abd.json')); c=d['config']['device_leg']
print('$v', round(d['value_device']/1e9,3), round(c['ms_per_step'],2), c['stage_ms_per_step'], c['counters_per_step']['n_records'])"
done
