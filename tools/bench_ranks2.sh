# Rehearsal of the driver's N>1 bench launch on a one-GPU box: two ranks share device 0.
# Default: `bench.py --gpus 2` alone (bench.py spawns its two ranks itself);
# LAUNCHER=torchrun: the driver's own torch.distributed.run command line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r04}
if [ "${LAUNCHER:-self}" = torchrun ]; then
  CMD=(python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py)
else
  CMD=(python bench.py)
fi
timeout -k 10 500 "${CMD[@]}" --gpus 2 --steps 3 --warmup 1 --reads 25000 --no-brand --cmr-steps 1 > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { tail -30 gpurun_out/bench2_$TAG.err; exit 1; }
cat gpurun_out/bench2_$TAG.json
