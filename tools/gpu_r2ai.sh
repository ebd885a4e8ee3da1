#!/bin/bash
# Round 2 (ai): A/B of the ring2 weight cache policy (nontemporal vs normal) at the bench default, interleaved.
set -o pipefail
mkdir -p gpurun_out/r2ai
for i in 1 2; do for nt in 1 0; do
  EDGELLM_TUNE="weight_nt=$nt" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-point off > gpurun_out/r2ai/nt${nt}_$i.log 2>&1 || { tail -5 gpurun_out/r2ai/nt${nt}_$i.log; exit 1; }
  tail -1 gpurun_out/r2ai/nt${nt}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('weight_nt', $nt, d['value'], d['p50_token_latency_ms'])"
done; done
