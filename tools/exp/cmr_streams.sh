#!/bin/bash
# create_mega_reads walls on 50k C2 reads by aligners per GPU (--streams), 3 cold runs each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for S in "$@"; do
  echo "== --streams $S"
  bash tools/exp/cmr_repeat.sh 50000 3 --streams $S | sed -e 's/"read_s.*"writer_idle_s": [0-9.]*, //' || exit 1
done
