#!/bin/bash
# Round 2 (m): prefill INT8 GEMM ring kernel — exactness/numerics tests, then the form sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "prefill_layout_exact or prefill_gemm or mfma_i8_layout or test_w8a8_gemm" > gpurun_out/r2m_tests.log 2>&1 || { tail -30 gpurun_out/r2m_tests.log; exit 1; }
tail -3 gpurun_out/r2m_tests.log
timeout -k 10 500 python -u tools/bench_ops.py --only pgemm --out gpurun_out/r2m_pgemm.json > gpurun_out/r2m_pgemm.log 2>&1
rc=$?; cat gpurun_out/r2m_pgemm.log | grep -v amdgpu.ids; exit $rc
