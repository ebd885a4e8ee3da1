#!/bin/bash
# Round 2 (af): multi-stage rehearsal on one GPU — 2 and 4 gloo ranks sharing the device (host-staged P2P), default config.
set -o pipefail
mkdir -p gpurun_out/r2af
for n in 2 4; do
  EDGELLM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2950$n bench.py --gpus $n --steps 12 --warmup 3 > gpurun_out/r2af/n$n.log 2>&1 || { tail -20 gpurun_out/r2af/n$n.log; exit 1; }
  grep '"metric"' gpurun_out/r2af/n$n.log | tail -1
done
