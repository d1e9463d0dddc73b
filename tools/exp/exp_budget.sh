set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 1.2e9 1.8e9 3.7e9; do
  timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline --no-brand --hit-budget $b > gpurun_out/budget_$b.json 2>gpurun_out/budget_$b.err || { tail -20 gpurun_out/budget_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/budget_$b.json'));print('$b',d['ms_per_step'],d['config']['stage_ms_per_step'])"
done
