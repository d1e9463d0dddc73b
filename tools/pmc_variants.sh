#!/bin/bash
# TCC hit/miss per k_coords launch for library variants (tools/exp/exp_coords.py).
# Usage (via gpurun): bash tools/pmc_variants.sh v1 v2 ...   (libpbgpu_<v>.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
  D=gpurun_out/pmcv_$v
  mkdir -p $D
  PBGPU_LIB=pacbio_amd/libpbgpu_$v.so timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_coords \
    --output-format csv -d $D -o run -- python3 tools/exp/exp_coords.py --reps 1 > $D/log 2>&1 || { tail -20 $D/log; exit 1; }
  python3 - "$D" "$v" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); disp = collections.defaultdict(set)
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "k_coords" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
print(sys.argv[2], {k: f"{v / len(disp[k]) / 1e6:.1f}M" for k, v in acc.items()}, "launches", max(len(s) for s in disp.values()))
PY
done
