# 32x32x32 prefill GEMM: correctness, then A/B (with the 256-row k-rotation A/B)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4d; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prefill_x32_gpu.py > $D/t.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/bench_ops.py --only x32,rot --out $D/ab.json > $D/ab.log 2>&1
