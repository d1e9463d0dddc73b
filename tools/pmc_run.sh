cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 1 --warmup 0 --reads 10000 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/kt -o run -- $B > gpurun_out/pmc_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/p1 -o run -- $B > gpurun_out/pmc_p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM --output-format csv -d gpurun_out/pmc/p2 -o run -- $B > gpurun_out/pmc_p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum --output-format csv -d gpurun_out/pmc/p3 -o run -- $B > gpurun_out/pmc_p3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/p4 -o run -- $B > gpurun_out/pmc_p4.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/p5 -o run -- $B > gpurun_out/pmc_p5.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc MeanOccupancyPerActiveCU --output-format csv -d gpurun_out/pmc/p6 -o run -- $B > gpurun_out/pmc_p6.log 2>&1
