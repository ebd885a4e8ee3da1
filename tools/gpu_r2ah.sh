#!/bin/bash
# Round 2 (ah): micro-batch size sweep above the 128-row fused path (one weight read per step for 256 rows).
set -o pipefail
mkdir -p gpurun_out/r2ah
for cfg in "1 256" "2 192" "1 192"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --lanes $1 --micro-batch $2 --steps 16 --warmup 4 --latency-point off > gpurun_out/r2ah/l$1_b$2.log 2>&1 || { tail -5 gpurun_out/r2ah/l$1_b$2.log; exit 1; }
  tail -1 gpurun_out/r2ah/l$1_b$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes', $1, 'mb', $2, d['value'], d['p50_token_latency_ms'])"
done
