#!/bin/bash
# Presence-filter A/B on the C2 bench (PBGPU_FILTER_BITS = bits per k-mer, 0 = off), after the GPU suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_filt.log 2>&1 || { tail -40 gpurun_out/gpu_tests_filt.log; exit 1; }
tail -2 gpurun_out/gpu_tests_filt.log
for b in ${BITS:-16 0 8 32}; do
  PBGPU_FILTER_BITS=$b timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline --no-brand > gpurun_out/filt_$b.json 2>gpurun_out/filt_$b.err || { tail -20 gpurun_out/filt_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/filt_$b.json'));c=d['config'];print('bits $b',round(d['ms_per_step'],2),c['stage_ms_per_step'],c['counters_per_step']['n_probes'],d['roofline']['kernel'],round(d['roofline']['frac'],3))"
done
