# Round 5: 8-rank gloo rehearsal of the N = 8 bench path on one GPU (per-stage calibration: each
# rank builds only its 4 layers; 64-row micro-batches so eight stages' caches fit one GPU)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5c; mkdir -p $D
EDGELLM_DIST_BACKEND=gloo timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 8 --steps 4 --warmup 2 --micro-batch 64 --latency-point off > $D/w8.log 2>&1 || exit $?
