#!/bin/bash
# Round 6: a.sh (tests, the C4 leg, its kernel trace), then the PMC calibration (pmc_group.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r06/a.sh || exit 1
bash tools/r06/pmc_group.sh
