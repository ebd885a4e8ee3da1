# Round-4: the pipeline path with the 2-lane default: RCCL at world 1 (--force-pipeline) and the
# 2-rank gloo rehearsal on one GPU at slack 0 / 1
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4q; mkdir -p $D
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --force-pipeline --latency-point off > $D/force_pp.log 2>&1 || exit $?
for SL in 0 1; do
  EDGELLM_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29610 + SL)) bench.py --gpus 2 --steps 12 --warmup 3 \
    --pp-slack $SL --latency-point off > $D/slack$SL.log 2>&1 || exit $?
done
