#!/bin/bash
# SQ counters of k_graph_edges (C2 50k reads, tools/prof_graph_gpu.py), one --pmc pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/edges_sq; rm -rf $D; mkdir -p $D
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES --kernel-include-regex "k_graph_edges<false" --output-format csv -d $D -o run -- python3 tools/prof_graph_gpu.py --reads 50000 > $D/log 2>&1 || { tail -20 $D/log; exit 1; }
python3 - "$D" <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(float); disp = set()
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        vals[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
for k, v in sorted(vals.items()): print(f"{k:20s} {v / max(1, len(disp)):.4g} per launch ({len(disp)} launches)")
PY
