# Round-4: 8-rank pipeline rehearsal on one GPU (gloo ranks sharing cuda:0, host-staged P2P): the
# N = 8 bench path end to end (half-layer stages, per-lane exchanges); 64-row micro-batches so
# eight stages' KV caches fit one GPU
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4z8; mkdir -p $D
EDGELLM_DIST_BACKEND=gloo timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 8 --steps 4 --warmup 2 --micro-batch 64 --latency-point off > $D/w8.log 2>&1 || exit $?
