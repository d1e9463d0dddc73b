#!/bin/bash
# e2e sweep of batch size / aligners per GPU (bench.py --no-cpu-baseline --no-brand)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 3 --device-steps 1 --no-cpu-baseline --no-brand --batch-bases $1 --streams $2 > gpurun_out/sweep_$1_$2.json 2>gpurun_out/sweep_$1_$2.err || { tail -5 gpurun_out/sweep_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sweep_$1_$2.json'));print('$1 $2', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['config']['stage_ms_per_step'])"
done
