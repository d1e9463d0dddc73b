# round 5: the GPU test suite in two parts (the C5 and scale tests take minutes each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PART=${1:-a}
if [ "$PART" = a ]; then
  timeout -k 10 1150 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    --ignore=tests/test_gpu_c5.py --ignore=tests/test_gpu_scale.py > gpurun_out/r05_suite_a.log 2>&1
else
  timeout -k 10 1150 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_scale.py -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r05_suite_b.log 2>&1
fi
rc=$?
tail -5 gpurun_out/r05_suite_$PART.log
exit $rc
