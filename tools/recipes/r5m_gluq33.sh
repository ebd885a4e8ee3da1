# Round 5: quantising gate_up at 33-64 rows on ring2 — fused-path tests and the GLU timings
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5m; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_decode_numerics_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_ops.py --only glu --no-sweep --out $D/ops.json > $D/ops.log 2>&1 || exit $?
