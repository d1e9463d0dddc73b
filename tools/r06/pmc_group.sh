#!/bin/bash
# Round 6: FETCH_SIZE of k_group's exact access shape (tools/calib_group.py: pass 0's 4-B ids,
# pass 1's 8-B words, both) against the known sector counts; k_group's FETCH / WRITE on C2
# (50k reads) with and without the 4-B super-read side array (PBGPU_OCC_SR=1) and on C4
# (the full index, 50k reads); SQ counters of k_coords and k_lis_w on C2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06b; mkdir -p $O
pm() {  # pm NAME COUNTER REGEX cmd...
  local n=$1 c=$2 re=$3; shift 3
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$re" --output-format csv -d $O/$n -o run -- "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; return 1; }
}
timeout -k 10 120 python3 -u tools/calib_group.py > $O/calib_group.json 2>&1 || exit 1
cat $O/calib_group.json
pm calib_fetch FETCH_SIZE k_gather_group python3 -u tools/calib_group.py || exit 1

for osr in 0 1; do
  if [ $osr = 1 ]; then export PBGPU_OCC_SR=1; fi
  timeout -k 10 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000 > $O/c2_time_osr$osr.txt 2>&1 || exit 1
  pm c2_fetch_osr$osr FETCH_SIZE k_group python3 -u tools/prof_lis.py --workload C2 --reads 50000 || exit 1
  pm c2_write_osr$osr WRITE_SIZE k_group python3 -u tools/prof_lis.py --workload C2 --reads 50000 || exit 1
  unset PBGPU_OCC_SR
done
bash tools/pmc_sq_any.sh "k_coords|k_lis_w" $O/sq_c2 -- python3 tools/prof_lis.py --workload C2 --reads 50000 > $O/sq_c2.txt 2>&1 || exit 1
for osr in 0 1; do
  if [ $osr = 1 ]; then export PBGPU_OCC_SR=1; fi
  timeout -k 10 400 python3 -u bench.py --only c4 --c4-reads 50000 --device-steps 2 > $O/c4_osr$osr.json 2>&1 || exit 1
  pm c4_fetch_osr$osr FETCH_SIZE k_group python3 -u bench.py --only c4 --c4-reads 50000 --no-brand --device-steps 1 || exit 1
  pm c4_write_osr$osr WRITE_SIZE k_group python3 -u bench.py --only c4 --c4-reads 50000 --no-brand --device-steps 1 || exit 1
  unset PBGPU_OCC_SR
done
python3 - $O <<'PY'
import csv, glob, sys, collections, os
O = sys.argv[1]
for d in sorted(glob.glob(O + "/*/")):
    acc = collections.defaultdict(list)
    for p in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            acc[(r.get("Kernel_Name", "?")[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{os.path.basename(d.rstrip('/')):18s} {k[0]:60s} {k[1]:22s} n={len(v):3d} mean={sum(v)/len(v):.6g} " + " ".join(f"{x:.4g}" for x in v[:8]))
PY
