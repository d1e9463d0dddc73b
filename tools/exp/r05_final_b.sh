# round 5: GPU suite part b, then the full-size device == host graph comparison
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/exp/r05_suite.sh b && bash tools/exp/r05_full_cmp.sh
