#!/bin/bash
# Round 2 (aj): lanes sweep at 128 rows on the round-2 kernels.
set -o pipefail
mkdir -p gpurun_out/r2aj
for l in 3 4; do
  timeout -k 10 300 python bench.py --lanes $l --steps 20 --warmup 5 --latency-point off > gpurun_out/r2aj/l$l.log 2>&1 || { tail -5 gpurun_out/r2aj/l$l.log; exit 1; }
  tail -1 gpurun_out/r2aj/l$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes', $l, d['value'], d['p50_token_latency_ms'], d['peak_mem_gb'])"
done
