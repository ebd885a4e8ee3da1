# Round 5: RCCL self-peer P2P (asserted), the world-1 RCCL pipeline engine's host issue time per
# tick, and 2- / 4-rank gloo rehearsals of the N > 1 bench path on one GPU (per-stage SmoothQuant
# calibration, half-layer stages, host_issue_us_per_tick in per_rank)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5b; mkdir -p $D
timeout -k 10 240 python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_rccl_gpu.py > $D/rccl.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --force-pipeline --steps 10 --warmup 3 --latency-point off > $D/w1_rccl.log 2>&1 || exit $?
EDGELLM_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 6 --warmup 2 --latency-point off > $D/w2.log 2>&1 || exit $?
EDGELLM_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 4 --steps 6 --warmup 2 --latency-point off > $D/w4.log 2>&1 || exit $?
