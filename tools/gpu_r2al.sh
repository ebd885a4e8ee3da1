#!/bin/bash
# Round 2 (al): new ring2 defaults — ring / rows128 / model tests, then the default bench twice.
set -o pipefail
mkdir -p gpurun_out/r2al
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py tests/test_model_gpu.py > gpurun_out/r2al/tests.log 2>&1 || { tail -30 gpurun_out/r2al/tests.log; exit 1; }
tail -1 gpurun_out/r2al/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2al/bench_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r2al/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['p50_token_latency_ms'], d.get('latency_point', {}).get('w8a8_smoothquant'))"
done
