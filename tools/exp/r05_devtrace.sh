# round 5: kernel trace of one device-leg call (C2 50k reads, one aligner): launches and gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r05zr
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d ${O}_trace -- python3 tools/exp/device_leg_trace.py > ${O}_run.txt 2>&1 || { tail -20 ${O}_run.txt; exit 1; }
F=$(find ${O}_trace -name "*kernel_trace.csv" | head -1)
python3 tools/exp/device_leg_trace.py --parse "$F" > ${O}_timeline.txt 2>&1 || exit 1
rm -rf ${O}_trace
tail -3 ${O}_timeline.txt
