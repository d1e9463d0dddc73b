#!/bin/bash
# k_coords ms and SQ instruction counts per variant (compile-out breakdown of the fit kernel)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/exp/coords_parts.sh "$@" || exit 1
for v in "" "$@"; do
  echo "== SQ ${v:-base}"
  bash tools/pmc_sq_kernel.sh k_coords $v 2>&1 | grep -E "SQ_INSTS|SQ_WAVES|SQ_WAVE_CYCLES|SQ_BUSY|SQ_ACTIVE_INST_VALU|SQ_WAIT" || exit 1
done
