#!/bin/bash
# Round 2 (o): prefill GEMM final form — kernel + model tests, form sweep, default bench.
set -o pipefail
mkdir -p gpurun_out/r2o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_decode_numerics_gpu.py \
  > gpurun_out/r2o/tests.log 2>&1 || { tail -30 gpurun_out/r2o/tests.log; exit 1; }
tail -2 gpurun_out/r2o/tests.log
timeout -k 10 500 python -u tools/bench_ops.py --only pgemm --out gpurun_out/r2o/pgemm.json > gpurun_out/r2o/pgemm.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r2o/bench.log 2>&1 || { tail -20 gpurun_out/r2o/bench.log; exit 1; }
grep metric gpurun_out/r2o/bench.log
