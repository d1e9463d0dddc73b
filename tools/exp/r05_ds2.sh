# round 5: graph tests with the 1024-record relax threshold; device leg with 1 and 2 aligners; cmr C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zg
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for s in 1 2 1 2; do
  timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --device-steps 5 --device-streams $s --cmr-steps 3 --parts 0 --c4r-reads 0 --no-cpu-baseline --skip-default-leg > ${O}_ds$s.json 2>> ${O}_ds.err || exit 1
  python3 -c "
import json; d=json.loads(open('${O}_ds$s.json').read().strip().splitlines()[-1])
print('streams', $s, 'value_device', round(d['value_device']/1e9,3), 'cmr', round(d['value_create_mega_reads']/1e9,3), d['create_mega_reads_walls_s'])" >> ${O}_summary.txt
done
cat ${O}_summary.txt
