# Round-4: per-lane pipeline exchanges: GPU pipeline tests, RCCL world-1 bench, 2-rank gloo rehearsal
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4r; mkdir -p $D
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pipeline_gpu.py tests/test_rccl_gpu.py tests/test_multiproc_gpu.py > $D/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --force-pipeline --latency-point off > $D/force_pp.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/gen.log 2>&1 || exit $?
EDGELLM_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29620 bench.py --gpus 2 --steps 12 --warmup 3 --latency-point off > $D/slack0.log 2>&1 || exit $?
