#!/bin/bash
# Norm prologue at 1-4 decode rows: numerics, then interleaved A/B (gemv_norm=1 / 0) at micro-batch 1 and 4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_gpu.py \
  -k "gemv_norm or defers_norms" > gpurun_out/r3s_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
: > gpurun_out/r3s_ab.jsonl
for mb in 4 1; do
  for k in 1 0 1 0; do
    EDGELLM_TUNE="gemv_norm=$k" timeout -k 10 240 python bench.py --micro-batch $mb --steps 64 --warmup 8 \
      --latency-point off > gpurun_out/r3s_b.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r3s_b.log; exit 1; }
    grep '^{' gpurun_out/r3s_b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());d['ab_label']='micro-batch $mb gemv_norm=$k';print(json.dumps(d))" >> gpurun_out/r3s_ab.jsonl
    python -c "import json;d=[json.loads(l) for l in open('gpurun_out/r3s_ab.jsonl')][-1];print(d['ab_label'],d['value'],d.get('p50_token_latency_ms'),d.get('p90_token_latency_ms'))"
  done
done
echo DONE
