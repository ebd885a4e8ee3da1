#!/bin/bash
# Round 2 (aa): one-round-trip norm kernel + bf16 decode GEMV at 17-64 rows — tests, bf16 row sweep vs hipBLASLt, default bench.
set -o pipefail
mkdir -p gpurun_out/r2aa
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_model_gpu.py > gpurun_out/r2aa/tests.log 2>&1 || { tail -30 gpurun_out/r2aa/tests.log; exit 1; }
tail -1 gpurun_out/r2aa/tests.log
timeout -k 10 300 python -u tools/bench_ops.py --only bf16rows --out gpurun_out/r2aa/bf16rows.json > gpurun_out/r2aa/bf16rows.log 2>&1 || { tail -5 gpurun_out/r2aa/bf16rows.log; exit 1; }
grep "'op'" gpurun_out/r2aa/bf16rows.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2aa/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2aa/bench.log
