cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -x -v --timeout 120 --timeout-method thread > gpurun_out/edge.log 2>&1 || { tail -30 gpurun_out/edge.log; exit 1; }
tail -3 gpurun_out/edge.log
bash tools/exp_libs.sh b512 && PBGPU_GROUP_TINY=0 NO_TESTS=1 bash tools/exp_libs.sh
