# Round 5: 8 gloo ranks sharing one GPU through the N = 8 bench path with the vocab-split head, at
# the bench's 256-row micro-batch (1 lane: eight stages' KV caches fit one GPU); the JSON carries
# the modelled stage costs (stage_cost_spread) and every rank's host issue time per tick
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5i; mkdir -p $D
EDGELLM_DIST_BACKEND=gloo timeout -k 10 1000 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29671 bench.py --gpus 8 --lanes 1 --steps 3 --warmup 1 --latency-point off > $D/w8.log 2>&1 || exit $?
