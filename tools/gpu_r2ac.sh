#!/bin/bash
# Round 2 (ac): fragment-packed A for the prefill GEMM — exactness, prefill GEMM timing; batch-1 spread; 1024-token TTFT.
set -o pipefail
mkdir -p gpurun_out/r2ac
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" > gpurun_out/r2ac/tests.log 2>&1 || { tail -30 gpurun_out/r2ac/tests.log; exit 1; }
tail -1 gpurun_out/r2ac/tests.log
timeout -k 10 400 python -u tools/bench_ops.py --only pgemm --out gpurun_out/r2ac/pgemm.json > gpurun_out/r2ac/pgemm.log 2>&1 || { tail -5 gpurun_out/r2ac/pgemm.log; exit 1; }
grep "'op'" gpurun_out/r2ac/pgemm.log | python -c "
import sys, ast
for l in sys.stdin:
    d = ast.literal_eval(l.strip()); print(d['shape'], d['M'], {k: v for k, v in d.items() if k.endswith('_TOPs')})"
timeout -k 10 200 python bench.py --micro-batch 1 --lanes 1 --prompt-len 1024 --steps 32 --warmup 4 --latency-point off > gpurun_out/r2ac/ttft1024.log 2>&1 || exit $?
tail -1 gpurun_out/r2ac/ttft1024.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > gpurun_out/r2ac/b1_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/r2ac/b1_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b1', d['p50_token_latency_ms'], d['value'], d['ttft_ms'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-point off > gpurun_out/r2ac/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2ac/bench.log
