# 1-GPU, 2-rank gloo rehearsal of the RCCL pipeline (EDGELLM_DIST_BACKEND=gloo: two ranks share the
# one GPU, P2P host-staged): slack 0 (hop on the critical path) vs slack 1 (hop beside a tick).
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4c; mkdir -p $D
for SL in 0 1; do
  EDGELLM_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + SL)) bench.py --gpus 2 --steps 12 --warmup 3 \
    --pp-slack $SL --latency-point off > $D/slack$SL.log 2>&1 || exit $?
  grep '^{' $D/slack$SL.log >> $D/rehearsal.jsonl
done
