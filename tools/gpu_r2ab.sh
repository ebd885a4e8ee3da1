#!/bin/bash
# Round 2 (ab): batch-1 spread (3 runs) and TTFT of a 1024-token refiner-size prompt at batch 1.
set -o pipefail
mkdir -p gpurun_out/r2ab
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > gpurun_out/r2ab/b1_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r2ab/b1_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b1', d['p50_token_latency_ms'], d['value'], d['ttft_ms'])"
done
timeout -k 10 200 python bench.py --micro-batch 1 --lanes 1 --prompt-len 1024 --steps 32 --warmup 4 --latency-point off > gpurun_out/r2ab/ttft1024.log 2>&1 || exit $?
tail -1 gpurun_out/r2ab/ttft1024.log
