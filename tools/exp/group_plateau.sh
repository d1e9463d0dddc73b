#!/bin/bash
# Evidence for k_group's plateau (round-3 review #7): per variant -- the whole group stage
# (gonly), pass 0 alone (p0), pass 0's loads without the table (p0notab), both passes
# without the list stores (nostore) -- the tier-0 ms (tools/prof_lis.py, 25k C2 reads) and
# FETCH_SIZE / WRITE_SIZE per tier-0 launch (separate --pmc passes).  Variants from
# tools/exp/build_group_variants.py.  Summary: gpurun_out/group_plateau.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/group_plateau.txt; : > $OUT
for v in "$@"; do
  lib=pacbio_amd/libpbgpu_$v.so; [ "$v" = base ] && lib=pacbio_amd/libpbgpu.so
  PBGPU_LIB=$lib timeout -k 10 300 python -u tools/prof_lis.py --reads 25000 > gpurun_out/gp_$v.txt 2>&1 || { cat gpurun_out/gp_$v.txt; exit 1; }
  echo "== $v: $(grep k_group gpurun_out/gp_$v.txt)" | tee -a $OUT
  for C in FETCH_SIZE WRITE_SIZE; do
    D=gpurun_out/gp_${v}_$C; mkdir -p $D
    PBGPU_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "k_group<false, 256u>" --output-format csv \
      -d $D -o run -- python3 tools/prof_lis.py --reads 25000 > $D/log 2>&1 || { tail -20 $D/log; exit 1; }
    python3 - "$D" "$v" "$C" <<'PY' | tee -a $OUT
import csv, glob, sys
vals = {}
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
v = sorted(vals.values())
print(f"   {sys.argv[2]} {sys.argv[3]}: {len(v)} launches, per launch KiB: {[round(x) for x in v]}")
PY
  done
done
