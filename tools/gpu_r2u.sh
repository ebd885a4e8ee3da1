#!/bin/bash
# Round 2 (u): query-head split attention + tied-head GEMV — tests, then the batch-1 configs.
set -o pipefail
mkdir -p gpurun_out/r2u
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py tests/test_kernels_gpu.py tests/test_decode_numerics_gpu.py tests/test_model_gpu.py \
  > gpurun_out/r2u/tests.log 2>&1 || { tail -30 gpurun_out/r2u/tests.log; exit 1; }
tail -1 gpurun_out/r2u/tests.log
timeout -k 10 600 python -u tools/bench_reference_config.py > gpurun_out/r2u/refcfg.log 2>&1 || { tail -20 gpurun_out/r2u/refcfg.log; exit 1; }
grep -h '^{' gpurun_out/r2u/refcfg.log | cut -c1-260
EDGELLM_TUNE=decode_attn_gsplit=1 timeout -k 10 300 python -u tools/bench_reference_config.py --models llama-3.2-1b --modes none,w8a8_smoothquant > gpurun_out/r2u/refcfg_nosplit.log 2>&1 || exit 1
grep -h '^{' gpurun_out/r2u/refcfg_nosplit.log | cut -c1-260
timeout -k 10 300 python -u bench.py --model llama-3-8b --micro-batch 1 --lanes 1 --steps 128 --warmup 8 --latency-point off > gpurun_out/r2u/l3_b1.log 2>&1 || exit 1
grep -h '^{' gpurun_out/r2u/l3_b1.log | cut -c1-300
