# Round-4 validation after the per-lane pipeline: full GPU suite, 2-rank rehearsal (slack 0 / 1), default bench
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4s; mkdir -p $D
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/gputest.log 2>&1 || exit $?
for SL in 0 1; do
  EDGELLM_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29630 + SL)) bench.py --gpus 2 --steps 12 --warmup 3 \
    --pp-slack $SL --latency-point off > $D/slack$SL.log 2>&1 || exit $?
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?
