# Round 5, final tree: gloo rehearsals of the N > 1 bench path on one GPU (ranks share cuda:0):
# 4 ranks at the default 2 x 256 lanes, 8 ranks at 1 lane of 256 rows (vocab-split head, per-stage calibration)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zf; mkdir -p $D
EDGELLM_DIST_BACKEND=gloo timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29691 bench.py --gpus 4 --steps 3 --warmup 1 --latency-point off > $D/w4.log 2>&1 || exit $?
EDGELLM_DIST_BACKEND=gloo timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29692 bench.py --gpus 8 --lanes 1 --steps 3 --warmup 1 --latency-point off > $D/w8.log 2>&1 || exit $?
