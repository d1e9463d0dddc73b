#!/bin/bash
# SQ instruction-mix passes over a short bench run (per-kernel LDS/VALU/VMEM mix).
set -o pipefail
TAG=${1:-sq}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/pmc_$TAG
mkdir -p $D
B="python3 bench.py --steps 1 --warmup 0 --reads 10000 --no-cpu-baseline --no-brand"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/kt -o run -- $B > $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH --output-format csv -d $D/p1 -o run -- $B > $D/p1.log 2>&1 || { tail -20 $D/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $D/p2 -o run -- $B > $D/p2.log 2>&1 || { tail -20 $D/p2.log; exit 1; }
echo done
