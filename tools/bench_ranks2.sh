# Rehearsal of the driver's N>1 bench launch on a one-GPU box: two ranks share device 0.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --reads 25000 --no-brand > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { tail -30 gpurun_out/bench2_$TAG.err; exit 1; }
cat gpurun_out/bench2_$TAG.json
