set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --reads 25000 --no-brand > gpurun_out/bench2_r01n.json 2> gpurun_out/bench2_r01n.err || { tail -30 gpurun_out/bench2_r01n.err; exit 1; }
cat gpurun_out/bench2_r01n.json
