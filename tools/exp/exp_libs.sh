#!/bin/bash
# GPU suite on the product library, then the C2 bench (3 steps) for it and each
# experiment variant libpbgpu_<name>.so given as arguments.
# Usage (via gpurun): bash tools/exp/exp_libs.sh [variant ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_exp.log 2>&1 || { tail -40 gpurun_out/gpu_tests_exp.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_exp.log
fi
for v in product "$@"; do
  L=pacbio_amd/libpbgpu.so; [ "$v" != product ] && L=pacbio_amd/libpbgpu_$v.so
  PBGPU_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline --no-brand > gpurun_out/exp_$v.json 2>gpurun_out/exp_$v.err || { tail -20 gpurun_out/exp_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp_$v.json'));c=d['config'];print('$v',round(d['ms_per_step'],2),c['stage_ms_per_step'],c['kernel_ms_per_launch'])"
done
