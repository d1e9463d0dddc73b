#!/bin/bash
# SQ counters of one kernel (regex) over tools/exp/exp_coords.py, two passes.
# Usage (via gpurun): bash tools/pmc_sq_kernel.sh REGEX [variant]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
RE=${1:-k_coords}; V=${2:-}
LIB=pacbio_amd/libpbgpu${V:+_$V}.so
D=gpurun_out/sqk_${RE}${V:+_$V}
mkdir -p $D
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  PBGPU_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RE" --output-format csv -d $D/p$i -o run -- \
    python3 tools/exp/exp_coords.py --reps 1 > $D/p$i.log 2>&1 || { tail -20 $D/p$i.log; exit 1; }
done
python3 - "$D" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); disp = collections.defaultdict(set)
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(acc):
    print(f"{k:24s} {acc[k] / len(disp[k]):14.4g} per launch")
PY
