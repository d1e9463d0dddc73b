#!/bin/bash
# Round 6, first GPU call: the records sort rewrite + overflow-list fix against the oracle
# (edge tests, C4r oracle parity), then the C4 leg alone and its kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06a
O=gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py "tests/test_gpu_configs.py::test_c4_repeat_model_oracle" \
  -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -8 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --only c4 --c4-reads 250000 > $O/c4.json 2> $O/c4.err
rc=$?; head -c 3000 $O/c4.json; tail -5 $O/c4.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o c4 -- python3 -u bench.py --only c4 --c4-reads 250000 --no-brand --device-steps 2 > $O/c4_prof.json 2> $O/c4_prof.err
rc=$?; tail -3 $O/c4_prof.err; exit $rc
