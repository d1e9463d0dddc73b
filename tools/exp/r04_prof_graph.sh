#!/bin/bash
# rocprofv3 kernel stats of the create_mega_reads device graph (tools/prof_graph_gpu.py, C2 reads)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-g}; N=${2:-50000}
D=gpurun_out/profg_$TAG; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/prof_graph_gpu.py --reads $N --workload ${WL:-C2} > $D/run.log 2>&1 || { tail -20 $D/run.log; exit 1; }
tail -3 $D/run.log
f=$(find $D -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:60]:60s} n={int(r["Calls"]):5d} total={float(r["TotalDurationNs"])/1e6:9.3f} ms avg={float(r["AverageNs"])/1e6:8.3f} ms')
PY
