# Round 5: LM head split by vocabulary over the pipeline ranks — GPU kernels (shard phase 1 + merge
# against the unsplit fused sampler), gloo ranks sharing the GPU (tokens equal the unsplit model's),
# then gloo rehearsals of the bench path at the bench's 256-row micro-batch: 4 ranks x 2 lanes and
# 8 ranks x 1 lane (memory: 8 stages' KV caches share one GPU), with the modelled stage costs
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5h; mkdir -p $D
[ -n "$SKIP_TESTS" ] || timeout -k 10 480 python -u -m pytest tests/test_vocab_split_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit $?
EDGELLM_DIST_BACKEND=gloo timeout -k 10 540 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29661 bench.py --gpus 4 --steps 4 --warmup 2 --latency-point off > $D/w4.log 2>&1 || exit $?
