# round 5: the mega-reads GPU tests (with the new many-batch host-read case)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mega_reads.py > gpurun_out/r05zo_tests.log 2>&1 || { tail -40 gpurun_out/r05zo_tests.log; exit 1; }
tail -1 gpurun_out/r05zo_tests.log
