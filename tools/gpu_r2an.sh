#!/bin/bash
# Round 2 (an): attention occupancy knob A/B in-model (interleaved), then 1-lane x 128 on the final defaults.
set -o pipefail
mkdir -p gpurun_out/r2an
for i in 1 2; do for t in "decode_attn_occ=4" "decode_attn_occ=5"; do
  n=$(echo $t | tr '=,' '__')
  EDGELLM_TUNE="$t" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-point off > gpurun_out/r2an/${n}_$i.log 2>&1 || { tail -5 gpurun_out/r2an/${n}_$i.log; exit 1; }
  tail -1 gpurun_out/r2an/${n}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['p50_token_latency_ms'])"
done; done
timeout -k 10 300 python bench.py --lanes 1 --steps 20 --warmup 5 --latency-point off > gpurun_out/r2an/l1.log 2>&1 || exit $?
tail -1 gpurun_out/r2an/l1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes 1', d['value'], d['p50_token_latency_ms'])"
