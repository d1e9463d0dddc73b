# round 5: SQ counters of the group kernels on C4r reads; the short-strand LIS tier A/B on C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/pmc_sq_any.sh "k_group" gpurun_out/r05p_sq -- python3 tools/prof_lis.py --workload C4r --reads 20000 > gpurun_out/r05p_sq.txt 2>&1 || exit 1
for e in 0 1; do
  echo "== PBGPU_LISW_SHORT=$e" >> gpurun_out/r05p_lisw.txt
  PBGPU_LISW_SHORT=$e timeout -k 10 300 python -u tools/prof_lis.py --workload C2 --reads 50000 >> gpurun_out/r05p_lisw.txt 2>&1 || exit 1
  PBGPU_LISW_SHORT=$e timeout -k 10 300 python -u tools/prof_lis.py --workload C4r --reads 20000 >> gpurun_out/r05p_lisw.txt 2>&1 || exit 1
done
PBGPU_LISW_SHORT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_regress.py > gpurun_out/r05p_tests.log 2>&1
tail -1 gpurun_out/r05p_tests.log
