#!/bin/bash
# Round 2 (ak): in-model A/B of the ring2 geometry / k-rotation (cfg 1, no rotation) at the bench default, interleaved.
set -o pipefail
mkdir -p gpurun_out/r2ak
for i in 1 2; do for t in "ring2_cfg=0,1" "ring2_cfg=1,0"; do
  n=$(echo $t | tr '=,' '__')
  EDGELLM_TUNE="$t" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-point off > gpurun_out/r2ak/${n}_$i.log 2>&1 || { tail -5 gpurun_out/r2ak/${n}_$i.log; exit 1; }
  tail -1 gpurun_out/r2ak/${n}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['p50_token_latency_ms'])"
done; done
