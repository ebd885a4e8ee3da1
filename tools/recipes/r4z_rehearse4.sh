# Round-4: 4-rank pipeline rehearsal on one GPU (gloo ranks sharing cuda:0, host-staged P2P):
# the N = 4 bench path end to end with half-layer stages and per-lane exchanges
set -o pipefail
export PYTHONUNBUFFERED=1
D=${D:-gpurun_out/r4z}; mkdir -p $D
EDGELLM_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 4 --steps 6 --warmup 2 --latency-point off > $D/w4.log 2>&1 || exit $?
