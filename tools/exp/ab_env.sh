#!/bin/bash
# device-leg A/B of an environment switch: bash tools/exp/ab_env.sh "VAR=val" ...  ("" = none)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for e in "$@"; do
  env $e timeout -k 10 400 python bench.py --steps 1 --warmup 0 --device-steps 3 --parts 0 --cmr-steps 0 --no-cpu-baseline --skip-default-leg --no-brand > gpurun_out/abe.json 2> gpurun_out/abe.err || { tail -5 gpurun_out/abe.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/abe.json')); c=d['config']['device_leg']
print('$e', round(d['value_device']/1e9,3), round(c['ms_per_step'],2), c['stage_ms_per_step'])"
done
