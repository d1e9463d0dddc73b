#!/bin/bash
# e2e bench under environment variants: bash tools/sweep_env.sh "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python -u bench.py --steps 3 --device-steps 1 --no-cpu-baseline --no-brand > gpurun_out/sweepenv_$i.json 2>gpurun_out/sweepenv_$i.err || { tail -5 gpurun_out/sweepenv_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sweepenv_$i.json'));print('$cfg', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['config']['stage_ms_per_step'])"
done
