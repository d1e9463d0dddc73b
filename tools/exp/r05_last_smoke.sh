# round 5: smoke() and the graph / edge GPU tests on the final tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_last_smoke.log 2>&1 || { tail -20 gpurun_out/r05_last_smoke.log; exit 1; }
tail -1 gpurun_out/r05_last_smoke.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_edge.py tests/test_gpu_parity.py > gpurun_out/r05_last_tests.log 2>&1 || { tail -30 gpurun_out/r05_last_tests.log; exit 1; }
tail -1 gpurun_out/r05_last_tests.log
