#!/bin/bash
# k_group tier 0 with fewer blocks a CU (PBGPU_GROUP_LDS_PAD bytes of extra dynamic LDS):
# tier-0 ms (tools/prof_lis.py, 25k C2 reads) and WRITE_SIZE per launch.  Does the list
# stores' write amplification follow the number of reads in flight?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/group_occupancy.txt; : > $OUT
for pad in "$@"; do
  PBGPU_GROUP_LDS_PAD=$pad timeout -k 10 300 python -u tools/prof_lis.py --reads 25000 > gpurun_out/go_$pad.txt 2>&1 || { cat gpurun_out/go_$pad.txt; exit 1; }
  echo "== pad $pad: $(grep k_group gpurun_out/go_$pad.txt | head -2 | tr '\n' ' ')" | tee -a $OUT
  D=gpurun_out/go_${pad}_W; mkdir -p $D
  PBGPU_GROUP_LDS_PAD=$pad timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_group<false, 256u>" --output-format csv \
    -d $D -o run -- python3 tools/prof_lis.py --reads 25000 > $D/log 2>&1 || { tail -20 $D/log; exit 1; }
  python3 - "$D" "$pad" <<'PY' | tee -a $OUT
import csv, glob, sys
vals = {}
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
v = sorted(vals.values())
print(f"   pad {sys.argv[2]} WRITE_SIZE: {len(v)} launches, per launch KiB: {[round(x) for x in v]}")
PY
done
