#!/bin/bash
# Round 6: new GPU tests; the C4 leg (250k reads) and its kernel trace; the group-shape
# PMC calibration; k_group FETCH/WRITE on C2 and C4 with and without the 4-B id side
# array; SQ counters of k_coords / k_lis_w on C2.
O=gpurun_out/r06c; mkdir -p gpurun_out/r06c
source tools/r06/lib.sh
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu"
step tests 900 $T tests/test_gpu_edge.py::test_group_first_round_items_overflow tests/test_gpu_mega_reads.py::test_device_graph_full_c4r_equals_host_graph tests/test_gpu_mega_reads.py::test_read_past_8192_records_against_restatement tests/test_gpu_mega_reads.py::test_device_graph_long_reads_c4r
step c4 500 python3 -u bench.py --only c4 --c4-reads 250000
head -c 2500 $O/c4.out; echo
step c4_trace 500 rocprofv3 --kernel-trace --stats -d $O/c4_trace -o c4 -- python3 -u bench.py --only c4 --c4-reads 100000 --no-brand --device-steps 1
pm() {  # pm NAME COUNTER REGEX cmd...
  local n=$1 c=$2 re=$3; shift 3
  step $n 300 rocprofv3 --pmc $c --kernel-include-regex "$re" --output-format csv -d $O/$n -o run -- "$@"
}
step calib 200 python3 -u tools/calib_group.py
cat $O/calib.out
pm calib_fetch FETCH_SIZE k_gather_group python3 -u tools/calib_group.py
for osr in 0 1; do
  if [ $osr = 1 ]; then export PBGPU_OCC_SR=1; fi
  step c2_time_osr$osr 300 python3 -u tools/prof_lis.py --workload C2 --reads 50000
  pm c2_fetch_osr$osr FETCH_SIZE k_group python3 -u tools/prof_lis.py --workload C2 --reads 50000
  pm c2_write_osr$osr WRITE_SIZE k_group python3 -u tools/prof_lis.py --workload C2 --reads 50000
  unset PBGPU_OCC_SR
done
step sq_c2 600 bash tools/pmc_sq_any.sh "k_coords|k_lis_w" $O/sq_c2 -- python3 tools/prof_lis.py --workload C2 --reads 50000
for osr in 0 1; do
  if [ $osr = 1 ]; then export PBGPU_OCC_SR=1; fi
  step c4_osr$osr 400 python3 -u bench.py --only c4 --c4-reads 50000 --device-steps 2 --no-brand
  pm c4_fetch_osr$osr FETCH_SIZE k_group python3 -u bench.py --only c4 --c4-reads 50000 --no-brand --device-steps 1
  pm c4_write_osr$osr WRITE_SIZE k_group python3 -u bench.py --only c4 --c4-reads 50000 --no-brand --device-steps 1
  unset PBGPU_OCC_SR
done
python3 - $O > $O/pmc_summary.txt <<'PY'
import csv, glob, sys, collections, os
O = sys.argv[1]
for d in sorted(glob.glob(O + "/*/")):
    acc = collections.defaultdict(list)
    for p in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            acc[(r.get("Kernel_Name", "?")[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{os.path.basename(d.rstrip('/')):18s} {k[0]:60s} {k[1]:22s} n={len(v):3d} mean={sum(v)/len(v):.6g} " + " ".join(f"{x:.4g}" for x in v[:12]))
PY
cat $O/steps.txt
