#!/bin/bash
# Round 2 (r): batch-1 launcher changes — attention/kernel tests, batch-1 latency, the reference's
# batch-1 configs (bf16 vs INT8), and a marker trace of the roctx ranges.
set -o pipefail
mkdir -p gpurun_out/r2r
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_decode_numerics_gpu.py tests/test_model_gpu.py \
  > gpurun_out/r2r/tests.log 2>&1 || { tail -30 gpurun_out/r2r/tests.log; exit 1; }
tail -1 gpurun_out/r2r/tests.log
timeout -k 10 300 python -u bench.py --micro-batch 1 --lanes 1 --steps 128 --warmup 8 --latency-point off > gpurun_out/r2r/b1_w8a8.log 2>&1 || exit 1
grep -h '^{' gpurun_out/r2r/b1_w8a8.log | cut -c1-400
timeout -k 10 300 python -u bench.py --quant none --micro-batch 1 --lanes 1 --steps 128 --warmup 8 --latency-point off > gpurun_out/r2r/b1_bf16.log 2>&1 || exit 1
grep -h '^{' gpurun_out/r2r/b1_bf16.log | cut -c1-400
timeout -k 10 600 python -u tools/bench_reference_config.py > gpurun_out/r2r/refcfg.log 2>&1 || { tail -20 gpurun_out/r2r/refcfg.log; exit 1; }
tail -12 gpurun_out/r2r/refcfg.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
EDGELLM_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/r2r/marker -- python3 bench.py --micro-batch 16 --lanes 1 --steps 8 --warmup 2 --latency-point off > gpurun_out/r2r/marker.log 2>&1 || { tail -10 gpurun_out/r2r/marker.log; exit 1; }
echo marker ok
