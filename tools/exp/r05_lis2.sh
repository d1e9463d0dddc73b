# round 5: LIS literal-step changes -- parity tests and stage times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zh
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_regress.py tests/test_gpu_edge.py > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for rep in 1 2; do
for wl in "C2 50000" "C4r 20000"; do
  set -- $wl
  timeout -k 10 300 python -u tools/prof_lis.py --workload $1 --reads $2 >> ${O}_stages.txt 2>&1 || exit 1
done
done
grep stages ${O}_stages.txt
