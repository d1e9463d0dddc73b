#!/bin/bash
# Round 6: the driver's N>1 launch rehearsed with 2 ranks on this 1-GPU box (ranks share the GPU;
# the C4 leg off: two 126-GB indexes do not fit one GPU)
O=gpurun_out/r06rh; mkdir -p gpurun_out/r06rh
source tools/r06/lib.sh
step bench2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --c4-reads 0
grep '^{"metric"' $O/bench2.out | head -c 1500; echo
cat $O/steps.txt
