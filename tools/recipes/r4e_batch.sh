# Round-4 validation batch: GPU tests (after pruning), x32 debug + tests, x32 prefill GEMM A/B,
# 256-row k-rotation A/B, default bench.
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4e; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
  --deselect tests/test_bf16_x32_gpu.py --deselect tests/test_prefill_x32_gpu.py > $D/gputest.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/x32_debug.py > $D/x32_debug.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_prefill_x32_gpu.py tests/test_bf16_x32_gpu.py > $D/x32_tests.log 2>&1
timeout -k 10 500 python3 tools/bench_ops.py --only rot --out $D/ab_rot.json > $D/ab_rot.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?
