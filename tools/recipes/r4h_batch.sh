# Round-4: 2 lanes x 256 rows, batch-1 weight-prefetch A/B, 1-GPU 2-rank gloo pipeline rehearsal
# (EDGELLM_PREFETCH, the batch-1 weight prefetch, measured slower here and was removed afterwards)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4h; mkdir -p $D
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --lanes 2 --latency-point off > $D/lanes2.log 2>&1 || exit $?
for PF in 0 1 3 11; do
  EDGELLM_PREFETCH=$PF timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --micro-batch 1 --latency-point off > $D/pf$PF.log 2>&1 || exit $?
done
for SL in 0 1; do
  EDGELLM_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + SL)) bench.py --gpus 2 --steps 12 --warmup 3 \
    --pp-slack $SL --latency-point off > $D/slack$SL.log 2>&1 || exit $?
done
