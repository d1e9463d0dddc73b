#!/bin/bash
# SQ counters of the kernels matching REGEX over any workload command, two passes, per kernel name.
# Usage (via gpurun): bash tools/pmc_sq_any.sh REGEX OUTDIR -- python3 tools/prof_lis.py --workload C4r --reads 20000
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
RE=$1; D=$2; shift 3
mkdir -p $D
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$RE" --output-format csv -d $D/p$i -o run -- "$@" > $D/p$i.log 2>&1 || { tail -20 $D/p$i.log; exit 1; }
done
python3 - "$D" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); disp = collections.defaultdict(set)
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = (r.get("Kernel_Name", "?")[:48], r["Counter_Name"])
        acc[k] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k in sorted(acc):
    print(f"{k[0]:48s} {k[1]:24s} {acc[k] / len(disp[k]):14.4g} per launch ({len(disp[k])} launches)")
PY
