#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/dev_kt; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O -o run -- python3 tools/exp/dev_trace.py > $O/out.log 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
cat $O/out.log
