# Round 5: vocab-split steps (shard, merge, penalty flags) captured in HIP graphs — GPU pipeline
# tests again, then the 8-rank gloo rehearsal at 256 rows (host issue time per tick)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5j; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py -k vocab -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit $?
EDGELLM_DIST_BACKEND=gloo timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29681 bench.py --gpus 8 --lanes 1 --steps 3 --warmup 1 --latency-point off > $D/w8.log 2>&1 || exit $?
