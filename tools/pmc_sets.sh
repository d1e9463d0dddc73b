#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, <= 8 SQ counters) for the kernels matching
# REGEX over tools/exp/exp_coords.py; prints the mean per launch.
# Usage (via gpurun): bash tools/pmc_sets.sh REGEX TAG "C1 C2 ..." ["C1 ..." ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
RE=$1; TAG=$2; shift 2
D=gpurun_out/pmcset_$TAG
mkdir -p $D
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RE" --output-format csv -d $D/p$i -o run -- \
    python3 tools/exp/exp_coords.py --reps 1 > $D/p$i.log 2>&1 || { tail -20 $D/p$i.log; exit 1; }
done
python3 - "$D" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); disp = collections.defaultdict(set)
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(acc):
    print(f"{k:28s} {acc[k] / len(disp[k]):14.4g} per launch")
PY
