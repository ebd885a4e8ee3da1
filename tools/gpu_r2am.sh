#!/bin/bash
# Round 2 (am): in-model sweep of the ring2 geometry knob (interleaved with the default).
set -o pipefail
mkdir -p gpurun_out/r2am
for t in "ring2_cfg=0,0" "ring2_cfg=2,0" "ring2_cfg=5,0" "ring2_cfg=0,0" "ring2_cfg=6,0" "ring2_cfg=3,0" "ring2_cfg=0,1"; do
  n=$(echo $t | tr '=,' '__')
  EDGELLM_TUNE="$t" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-point off > gpurun_out/r2am/$n.log 2>&1 || { tail -5 gpurun_out/r2am/$n.log; exit 1; }
  tail -1 gpurun_out/r2am/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['p50_token_latency_ms'])"
done
